#!/usr/bin/env python3
"""Time the REFERENCE's own placement functions (rescheduling.py:77-218) the way
tools/dropin_latency.py times the drop-in, and write the medians to
profiles/ref_latency_container.json.

Runs only in the build container: it imports /root/reference through the
test-side kubernetes stub (tests/stubs, as tests/golden/make_golden.py does) and
never travels to the GPU box.  Configs:

* ``wm3``   — the reference's own operating point (README.md:44-48): the µBench
  workmodelC services on 3 workers, replayed from the 103 three-worker snapshots
  of tests/golden/wm_snapshots.json (each call on the next snapshot);
* ``2k64``, ``100k5k`` — the synthetic clusters of SURVEY.md §8d (rsk/synth.py).

    python -B tools/ref_latency.py [--ref /root/reference] [--calls 50]
"""
import argparse
import copy
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests", "stubs"), os.path.join(REPO, "kubernetes-rescheduling_amd")]
sys.path.insert(0, os.path.join(REPO, "tools"))

ALGOS = ("communication", "spread", "binpack", "random")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "ref_latency_container.json"))
    args = ap.parse_args()
    sys.path.insert(0, args.ref)  # ahead of the package dir: its rescheduling.py is the drop-in
    import numpy as np
    import rescheduling as R  # the reference module
    assert os.path.dirname(os.path.abspath(R.__file__)) == os.path.abspath(args.ref), R.__file__
    from kubernetes import client
    from dropin_latency import cases
    rows = []
    for cfg, case_iter in cases(args.calls):
        for algo in ALGOS:
            times = []
            for k, (info, hz, cm, rel, names) in enumerate(case_iter()):
                client.CREATED.clear()
                random.seed(k)
                t0 = time.perf_counter()
                try:
                    if algo == "communication":
                        R.communication(info, hz, cm, rel, names)
                    elif algo == "spread":
                        R.spread(info, hz, cm)
                    elif algo == "binpack":
                        R.binpack(info, hz, cm)
                    else:
                        R.random(info, hz, names)
                except (RuntimeError, ValueError):
                    pass
                dt = (time.perf_counter() - t0) * 1e3
                if k >= 3:
                    times.append(dt)
            t = np.array(times)
            row = {"config": cfg, "algo": algo, "calls": len(t), "median_ms": round(float(np.median(t)), 4),
                   "p90_ms": round(float(np.percentile(t, 90)), 4)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    cpu = "unknown"
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    with open(args.out, "w") as f:
        json.dump({"host": f"build container, 1 core of {os.cpu_count()} ({cpu})", "python": sys.version.split()[0],
                   "method": "reference rescheduling.py through tests/stubs, same call sequence as "
                             "tools/dropin_latency.py (create() hits the stub)", "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
