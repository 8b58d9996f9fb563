"""Host cost of one CAR step (plan.execute through ctypes) against its device
time, at a bench config: if the host needs about as long per call as the GPU
per step, the step is host-bound and the kernels wait between launches.
usage: python tools/hostprobe.py [headline|1m50k]"""
import json
import os
import sys
import time

REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [os.path.join(REPO, "kubernetes-rescheduling_amd"), REPO]

import torch  # noqa: E402
from rsk import _lib, api, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "1m50k"
P, N, S = {"headline": (100_000, 5_000, 4096), "1m50k": (1_000_000, 50_000, 64)}[cfg]
c = synth.make_cluster(P, N, S=S, seed=0)
dev = torch.device("cuda:0")
ctx = _lib.Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
plan = api.CarPlan(c.row_ptr, c.col_idx, ctx=ctx)
T = {k: torch.from_numpy(getattr(c, k)).to(dev) for k in ("assign", "cap_cpu", "use_cpu", "hazard")}
out = torch.empty(P * S, dtype=torch.int32, device=dev)
args = (T["assign"], S, T["cap_cpu"], T["use_cpu"], T["hazard"], N, out, None)
for _ in range(5):
    plan.execute(*args, device=True)
torch.cuda.synchronize(dev)
res = {"config": cfg}
for steps in (1, 5, 20):
    host = []
    t0 = time.perf_counter()
    for _ in range(steps):
        h = time.perf_counter()
        plan.execute(*args, device=True)
        host.append(time.perf_counter() - h)
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    res[f"steps{steps}"] = {"host_us_per_call": round(sum(host) / steps * 1e6, 1),
                            "enqueue_us": round((t1 - t0) * 1e6, 1),
                            "wall_us_per_step": round((t2 - t0) / steps * 1e6, 1)}
print(json.dumps(res), flush=True)
