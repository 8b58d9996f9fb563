#!/usr/bin/env python3
"""Headline CAR step alone, for PMC passes of experiment libraries.

bench.py refuses the wrong-result profiling ablations (RSK_ABLATE_*); this
tool runs the same config-3 batch (or --config 1m50k) through
rsk_car_plan_execute --steps times with no parity check, so a rocprofv3 --pmc
pass can read an ablation's FETCH_SIZE / WRITE_SIZE (RSK_LIB=.../librsk_abl.so
RSK_ABLATE_TILE=8: every code gather from one line — the code-line traffic by
difference).  Prints one line: ms per step (wall clock, device-synchronised).
"""
import argparse
import os
import sys
import time

REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "kubernetes-rescheduling_amd"), REPO]

CFG = {"headline": (100_000, 5_000, 4096), "1m50k": (1_000_000, 50_000, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="headline", choices=sorted(CFG))
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import torch
    from rsk import _lib, api, synth
    P, N, S = CFG[args.config]
    dev = torch.device("cuda", 0)
    c = synth.make_cluster(P, N, S=S, seed=0)
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    plan = api.CarPlan(c.row_ptr, c.col_idx, ctx=ctx)
    T = {k: torch.from_numpy(getattr(c, k)).to(dev) for k in ("assign", "cap_cpu", "use_cpu", "hazard")}
    out = torch.empty(P * S, dtype=torch.int32, device=dev)

    def step():
        plan.execute(T["assign"], S, T["cap_cpu"], T["use_cpu"], T["hazard"], N, out, None, device=True)

    step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3 / args.steps
    env = {k: v for k, v in os.environ.items() if k.startswith("RSK_")}
    print(f"tilebench {args.config} ms_per_step {ms:.4f} env {env}", flush=True)
    plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
