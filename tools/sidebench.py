"""Config-4 (1M pods x 50k nodes x 64 scenarios) CAR step with librsk's kernel
timers: per-kernel averages and the step time, for A/B of library variants
(RSK_LIB=.../librsk_<variant>.so; an ablation build takes RSK_ABLATE_SIDE /
RSK_ABLATE_TILE here — bench.py refuses those).  Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [os.path.join(REPO, "kubernetes-rescheduling_amd"), REPO]

import torch  # noqa: E402
from rsk import _lib, api, synth  # noqa: E402

P, N, S = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (1_000_000, 50_000, 64)))
steps = 20
c = synth.make_cluster(P, N, S=S, seed=0)
dev = torch.device("cuda:0")
ctx = _lib.Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
plan = api.CarPlan(c.row_ptr, c.col_idx, ctx=ctx)
T = {k: torch.from_numpy(getattr(c, k)).to(dev) for k in ("assign", "cap_cpu", "use_cpu", "hazard")}
out = torch.empty(P * S, dtype=torch.int32, device=dev)


def step():
    plan.execute(T["assign"], S, T["cap_cpu"], T["use_cpu"], T["hazard"], N, out, None, device=True)


for _ in range(3):
    step()
torch.cuda.synchronize(dev)
t0 = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize(dev)
ms = (time.perf_counter() - t0) * 1e3 / steps
ctx.reset_profiling()
ctx.set_profiling(True)
for _ in range(steps):
    step()
torch.cuda.synchronize(dev)
ctx.set_profiling(False)
names = ("car_prep", "car_tile", "car_tile_heavy", "car_side", "car_side32", "car_side128", "car_side512",
         "car_side2048", "car_side8192", "car_side65535")
k = {}
for name in names:
    t, n = ctx.kernel_time(name)
    if n:
        k[name] = round(t / n, 4)
print(json.dumps({"P": P, "N": N, "S": S, "ms_per_step": round(ms, 4), "kernels": k,
                  "env": {a: b for a, b in os.environ.items() if a.startswith("RSK_")}}), flush=True)
