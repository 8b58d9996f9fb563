import os, sys, numpy as np
sys.path[:0] = ["kubernetes-rescheduling_amd", "."]
os.environ["RSK_ABLATE_PIVOT"] = "32"
from rsk import api, synth, _lib
c = synth.make_cluster(100000, 5000, S=4096, seed=0)
plan = api.CarPlan(c.row_ptr, c.col_idx)
import ctypes
t, _ = plan.execute(c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N)
deg = np.diff(c.row_ptr)
rows = np.nonzero(deg > 32)[0]
tt = t.reshape(c.P, c.S)[rows]
print("rows", len(rows), "delta per lane: mean", tt.mean(), "max", tt.max(), "ovf lanes", (tt >= 1000).sum())
for r in rows[:5]:
    print(r, deg[r], np.bincount(np.minimum(t.reshape(c.P,c.S)[r], 40))[:20])
