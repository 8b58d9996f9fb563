import sys, time, os
sys.path[:0] = [os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "kubernetes-rescheduling_amd")]
import numpy as np
from rsk import api
rng = np.random.default_rng(0)
for N, k in [(64, 40), (5000, 500), (5000, 5)]:
    node_of = rng.integers(0, N, k).astype(np.int32)
    cap = np.full(N, 64000, np.int32); use = rng.integers(0, 16000, N).astype(np.int32); haz = (rng.random(N) < 0.15).astype(np.uint8)
    rp = np.array([0, k] + [k] * k, np.int32); ci = np.arange(1, k + 1, dtype=np.int32); asg = np.concatenate([[-1], node_of]).astype(np.int32)
    for name, f in [("row", lambda: api.car_row(node_of, cap, use, haz, N)), ("place", lambda: api.car_place(rp, ci, asg, 1, cap, use, haz, N, rows=[0]))]:
        f()
        ts = []
        for _ in range(30):
            t0 = time.perf_counter(); f(); ts.append(time.perf_counter() - t0)
        print(N, k, name, "median_ms %.4f" % (np.median(ts) * 1e3), flush=True)
