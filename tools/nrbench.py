"""rsk_node_reduce at 1M pods x 50k nodes x 64 scenarios (bench.py's kernel-3
case) with librsk's timer: for A/B of library variants (RSK_LIB).  One JSON line."""
import json
import os
import sys
import time

REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [os.path.join(REPO, "kubernetes-rescheduling_amd"), REPO]

import torch  # noqa: E402
from rsk import _lib, synth  # noqa: E402

P, N, S = 1_000_000, 50_000, 64
c = synth.make_cluster(P, N, S=S, seed=0)
dev = torch.device("cuda:0")
ctx = _lib.Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
a, pc, pm = T(c.assign), T(c.pod_cpu), T(c.pod_mem)
cnt = torch.empty(N * S, dtype=torch.int32, device=dev)
cpu = torch.empty(N * S, dtype=torch.int64, device=dev)
mem = torch.empty(N * S, dtype=torch.int64, device=dev)


def call():
    _lib.check(ctx.lib.rsk_node_reduce(ctx.handle, a.data_ptr(), P, S, pc.data_ptr(), pm.data_ptr(), N,
                                       cnt.data_ptr(), cpu.data_ptr(), mem.data_ptr(), _lib.RSK_F_DEVICE))


for _ in range(3):
    call()
torch.cuda.synchronize(dev)
n = 20
t0 = time.perf_counter()
for _ in range(n):
    call()
torch.cuda.synchronize(dev)
wall = (time.perf_counter() - t0) * 1e3 / n
ctx.reset_profiling()
ctx.set_profiling(True)
for _ in range(n):
    call()
torch.cuda.synchronize(dev)
ctx.set_profiling(False)
ms, k = ctx.kernel_time("node_reduce")
ucap = T(c.cap_cpu)
use = T(c.use_cpu)
std = torch.empty(S, dtype=torch.float64, device=dev)
ctx.reset_profiling()
ctx.set_profiling(True)
for _ in range(n):
    _lib.check(ctx.lib.rsk_load_std(ctx.handle, use.data_ptr(), ucap.data_ptr(), N, S, std.data_ptr(),
                                    _lib.RSK_F_DEVICE))
torch.cuda.synchronize(dev)
ctx.set_profiling(False)
ms2, k2 = ctx.kernel_time("load_std")
print(json.dumps({"wall_ms": round(wall, 4), "node_reduce_ms": round(ms / max(k, 1), 4),
                  "load_std_ms": round(ms2 / max(k2, 1), 4),
                  "env": {x: y for x, y in os.environ.items() if x.startswith("RSK_")}}), flush=True)
