#!/usr/bin/env python3
"""Headline benchmark: CAR placement scoring, pod×node move evaluations / s.

Workload (BASELINE.json configs[2]): 100k pods, 5k
nodes, preferential-attachment relation tree, S = 4096 what-if scenarios per
GPU.  One step = one pass of the hot path over one batch: librsk's CAR pipeline
(car_prep, then the tiles fused with the side rows in one launch — car_tile —
and, at config 4, the largest side rows beside them on a second stream —
car_side) scores every pod in every scenario against every node — P·N·S
evaluations — with all inputs resident in HBM.

Secondary configs: with no ``--config`` the line also carries ``configs``:
config 2, config 4 (its CAR step, the row-sharded loop and kernel 3), config 5
and config 5 at its 8-GPU per-rank share (S = 128), each run after the
headline's timed region and parity sample with its own timing, parity check
and roofline (one GPU only; ``--no-extra`` skips them).

Multi-GPU: ``python bench.py --gpus N`` with no ``WORLD_SIZE`` in the
environment starts ``torch.distributed.run --nproc-per-node N`` on itself as a
child process (the parent touches no GPU) and exits with its status; under a
launcher (``WORLD_SIZE`` set) it must equal ``--gpus``.  Scenario sharding: rank
r scores global scenarios [r·S, (r+1)·S) with no data-path collective;
``value`` is the whole-job rate (weak scaling).  Timing: barrier + device sync
around exactly ``--steps`` steps, max over ranks.  Per-kernel times come from
HIP events on the stream the kernels run on (librsk's profiler).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "kubernetes-rescheduling_amd"), REPO]

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)

CONFIGS = {
    "headline": dict(P=100_000, N=5_000, S=4096, name="100k pods x 5k nodes, PA tree, 4096 scenarios/GPU (config 3)",
                     metric="pod×node move evaluations/sec at 100k pods×5k nodes; % of HBM roofline"),
    "2k64": dict(P=2_000, N=64, S=1, name="2k pods x 64 nodes, single CAR round (config 2)",
                 metric="pod×node move evaluations/sec at 2k pods×64 nodes, one CAR round (latency-bound)"),
    "rounds": dict(P=100_000, N=5_000, S=1024, rounds=True,
                   name="100k pods x 5k nodes x 1024 scenarios/GPU, detect -> evict -> CAR -> update rounds (config 5)",
                   metric="rescheduling rounds x scenarios per second (detect -> evict -> CAR -> update)"),
    "1m50k": dict(P=1_000_000, N=50_000, S=64, shard="rows",
                  name="1M pods x 50k nodes x 64 scenarios, pod-row sharded (config 4)",
                  metric="pod×node move evaluations/sec at 1M pods×50k nodes; % of HBM roofline"),
}
PMC_JSON = os.path.join(REPO, "profiles", "pmc_traffic.json")


def cpu_model():
    """Host CPU model name and logical CPU count (the GPU box's host cores)."""
    name = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return name, os.cpu_count() or 1


def cgroup_cpu_quota():
    """The cgroup v2 CPU limit as cores (cpu.max quota / period), None when unlimited or unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_threads():
    """Threads for the OpenMP CPU leg: the affinity mask capped by the cgroup's
    CPU quota (a quota of 16 cores on a 256-CPU host gives 16 threads)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpu_quota()
    return max(1, min(aff, math.ceil(quota))) if quota else aff, aff


# Environment knobs the benchmark records.  librsk.so reads none of them (its
# tuning switches exist only in `make variant` builds); an ablation variable
# means someone expected wrong-result switches, so no line is printed.
ABLATION_VARS = ("RSK_ABLATE_TILE", "RSK_ABLATE_SIDE")


def rsk_env():
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("RSK_")}


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`--gpus N` without a launcher: run N ranks of this script under
    torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) and return
    its exit status (non-zero when any rank fails).  Called before anything
    touches a GPU, so the parent never initialises HIP; rank 0 prints the line
    straight to the inherited stdout."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    log(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd, env=dict(os.environ))


def dry_run(args, world, rank):
    """`--dry-run`: the multi-rank skeleton on the CPU (gloo, no GPU, no librsk):
    rendezvous, the scenario shard of every rank, exactly --steps barrier-
    bracketed no-op steps, the MAX-over-ranks time, and rank 0's line naming
    every rank that took part.  tests/test_bench_launcher.py runs it at --gpus 2."""
    import torch
    import torch.distributed as dist
    from rsk import dist as rdist
    if world > 1:
        dist.init_process_group("gloo")
    S = CONFIGS[args.config]["S"]
    sh = rdist.shard_for(rank, world, S)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    mine = torch.tensor([rank, sh.s0, sh.s0 + sh.s_local, os.getpid()], dtype=torch.int64)
    rows = [mine]
    if world > 1:
        rows = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(rows, mine)
        e = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "rccl_world": dist.get_world_size() if world > 1 else 1,
                          "backend": "gloo" if world > 1 else None, "steps": args.steps,
                          "ranks": [int(r[0]) for r in rows], "pids": [int(r[3]) for r in rows],
                          "scenario_shards": [[int(r[1]), int(r[2])] for r in rows],
                          "ms_per_step": el * 1e3 / max(args.steps, 1), "env": rsk_env()}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def python_legs(c, N, S, budget_s=6.0, numpy_budget_s=20.0):
    """SURVEY §8d CPU legs 1 and 2 (oracle/car_py.py, one core): the literal
    pure-Python restatement of rescheduling.py:183-214 on 64 evenly spaced pods
    of scenario 0, and the numpy vectorized one on every pod of scenario 0.
    One call = one (pod, scenario) = N evaluations."""
    from oracle import car_py
    P = c.P
    pods = np.linspace(0, P - 1, 64).astype(np.int64)
    nbrs = car_py.dedup_rows(c.row_ptr, c.col_idx, pods)
    legs = []
    a, u, h = car_py.scenario_view(c.assign, c.use_cpu, c.hazard, P, N, S, 0)
    by_node = car_py.pods_by_node(a, N)
    haz_list = [n for n in range(N) if h[n]]
    t0 = time.perf_counter()
    calls = 0
    for nb in nbrs:
        car_py.car_literal(nb.tolist(), by_node, haz_list, c.cap_cpu, u)
        calls += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    legs.append({"kind": "port", "impl": "literal pure-Python restatement (oracle/car_py.car_literal)",
                 "value": round(calls * N / dt, 1), "unit": "pod×node evals/s", "cores": 1,
                 "sample": f"{calls} evenly spaced pods x scenario 0 x {N} nodes",
                 "ms_per_call": round(dt * 1e3 / calls, 3)})
    # leg 2 (BASELINE.md "CPU-baseline plan" item 2): every pod of scenario 0,
    # capped at numpy_budget_s (then the pods done are reported)
    nb_all = car_py.dedup_rows(c.row_ptr, c.col_idx, range(P))
    calls = 0
    t0 = time.perf_counter()
    for nb in nb_all:
        car_py.car_numpy(nb, a, c.cap_cpu, u, h, N)
        calls += 1
        if (calls & 255) == 0 and time.perf_counter() - t0 > numpy_budget_s:
            break
    dt = time.perf_counter() - t0
    legs.append({"kind": "port", "impl": "numpy vectorized restatement (oracle/car_py.car_numpy)",
                 "value": round(calls * N / dt, 1), "unit": "pod×node evals/s", "cores": 1,
                 "sample": f"{'all ' if calls == P else ''}{calls} of {P} pods x scenario 0 x {N} nodes",
                 "ms_per_call": round(dt * 1e3 / calls, 4)})
    return legs


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(P, N, S, nnz, Q_light=None, light_rec_bytes=0):
    """B = 4(P+1) + 4nnz + 4PS + 4N + 5NS + 4PS per batch."""
    return 4 * (P + 1) + 4 * nnz + 4 * P * S + 4 * N + 5 * N * S + 4 * P * S


def alg_bytes(kernel, P, N, S, info, step_bytes=0):
    """Algorithmic bytes per step of one kernel timer (DESIGN.md "Roofline accounting"):
      car_direct : the one-launch small batch (config 2): the whole step's SURVEY §8d bytes
      car_tile : the tile launch (tiles + the side rows fused into it): the assign slice of every
                 distinct neighbour pod of those rows once (4·S per pod) + every row's target (4·S)
                 + the tile plan and side items
      car_side : target of each side row launched on its own (4·S) + side items / neighbour lists
                 (its neighbours' slices: re-reads of pods the tiles stage, not counted)
      car_mid / car_heavy : the wide path's (N > 65535) side rows
      car_prep : use + hazard (5·N·S) + cap (4·N) read, the 16-bit code (2·N·S) written
    """
    fused = info.get("fused_side_rows", 0)
    nb = info.get("fused_nb_pods_distinct", info["image_pods_distinct"])
    return {"car_tile": 4 * S * nb + 4 * S * (info["tile_rows"] + fused) + info["tile_bytes"]
                        + (info.get("side_bytes", 0) if fused else 0),
            "car_side": 4 * S * (info.get("side_rows", 0) - fused) + info.get("side_bytes", 0),
            "car_mid": 4 * S * info["mid_rows"] + info["mid_bytes"],
            "car_heavy": 4 * S * info["heavy_rows"] + info["heavy_bytes"],
            "car_prep": 7 * N * S + 4 * N,
            "car_direct": step_bytes}.get(kernel, 0)


def bench_rounds(args, cfg, world, rank, local, dev):  # noqa: C901
    """Config 5: one step = one round of detect -> evict -> CAR -> update over
    this rank's S scenarios.  The timed region is ONE rsk_rounds_run call of R =
    --steps rounds (default 256, config 5's R) with the state on the device; the
    warm-up is another call of --warmup rounds from the same state.  Scenario
    sharded, no data-path collective."""
    import torch
    import torch.distributed as dist
    from rsk import _lib, api, synth
    from rsk import dist as rdist
    P, N, S = cfg["P"], cfg["N"], cfg["S"]
    shard = rdist.shard_for(rank, world, S)
    c = synth.make_cluster(P, N, S=S, seed=0, s0=shard.s0)
    ctx = _lib.Context(local)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    rounds = api.Rounds(c.row_ptr, c.col_idx, c.pod_cpu, ctx=ctx)
    T = {k: torch.from_numpy(np.ascontiguousarray(getattr(c, k), dtype=np.int32)).to(dev)
         for k in ("assign", "cap_cpu", "use_cpu")}
    R = args.warmup + args.steps
    ev = torch.empty(R * S, dtype=torch.int32, device=dev)
    tg = torch.empty(R * S, dtype=torch.int32, device=dev)
    if args.warmup:
        rounds.run(T["assign"], S, T["cap_cpu"], T["use_cpu"], N, args.warmup, 30, ev, tg, device=True)
    # the timed call's own starting state (parity of every scenario below)
    k = S
    a_start = T["assign"].view(P, S)[:, :k].cpu().numpy().copy().reshape(-1)
    u_start = T["use_cpu"].view(N, S)[:, :k].cpu().numpy().copy().reshape(-1)
    # the timed call runs without kernel events (an event pair around every
    # launch adds its own packets between the round's kernels); the per-kernel
    # breakdown comes from a separate call below
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    w = args.warmup * S
    rounds.run(T["assign"], S, T["cap_cpu"], T["use_cpu"], N, args.steps, 30, ev[w:], tg[w:], device=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t1
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    tgt = tg.cpu().numpy()[args.warmup * S:]
    # parity of the timed call itself: every scenario, all R rounds from the
    # state it started from, against oracle_rounds (final assign / use,
    # evictions and targets of every round; the scenarios split over threads)
    from oracle import oracle as orc
    R = args.steps
    t_par = time.perf_counter()
    ea, eu, eev, etg = orc.rounds(c.row_ptr, c.col_idx, c.pod_cpu, a_start, k, c.cap_cpu, u_start, N, R,
                                  threads=cpu_threads()[0])
    parity_s = time.perf_counter() - t_par
    got_ev = ev.cpu().numpy()[w:].reshape(R, S)[:, :k].reshape(-1)
    got_a = T["assign"].view(P, S)[:, :k].cpu().numpy().reshape(-1)
    got_u = T["use_cpu"].view(N, S)[:, :k].cpu().numpy().reshape(-1)
    parity_ok = bool(np.array_equal(tgt.reshape(R, S)[:, :k].reshape(-1), etg) and np.array_equal(got_ev, eev)
                     and np.array_equal(got_a, ea) and np.array_equal(got_u, eu))
    ms_step = elapsed * 1e3 / args.steps
    kernels = {}
    if not args.no_kernel_events:  # the breakdown: another call of the same R, events around every launch
        a_keep, u_keep = T["assign"].clone(), T["use_cpu"].clone()
        ctx.reset_profiling()
        ctx.set_profiling(True)
        rounds.run(T["assign"], S, T["cap_cpu"], T["use_cpu"], N, args.steps, 30, ev[w:], tg[w:], device=True)
        torch.cuda.synchronize(dev)
        ctx.set_profiling(False)
        T["assign"].copy_(a_keep)
        T["use_cpu"].copy_(u_keep)
        for name in ("rounds_lists", "rounds_detect", "rounds_persist"):
            ms, n = ctx.kernel_time(name)
            if n:
                kernels[name] = {"avg_ms": ms / n, "launches": n, "per_step_ms": ms / args.steps}
    line = None
    if rank == 0:
        line = {
            "metric": cfg["metric"],
            "value": round(world * S / (ms_step / 1e3), 1), "unit": "scenario-rounds/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": cfg["name"], "pods": P, "nodes": N, "scenarios_per_gpu": S, "threshold": 30,
                       "rounds_per_call": args.steps,
                       "parallelism": f"scenario-sharded x{world}"},
            "kernels": kernels,
            "kernels_note": "a separate call of the same R with HIP events around every launch (the timed call has none)",
            "moves": int((tgt >= 0).sum()), "none": int((tgt == -1).sum()),
            "no_candidate": int((tgt == -2).sum()), "no_evict": int((tgt == -3).sum()),
            "parity_sample_ok": bool(parity_ok),
            "parity_sample": f"the timed {R}-round call, all {k} scenarios (0..{k - 1}), vs oracle_rounds from its "
                             f"start state ({parity_s:.1f} s on {cpu_threads()[0]} threads)",
            "rccl_world": args.rccl_world, "env": rsk_env(),
        }
    rounds.close()
    ctx.close()
    return line if rank == 0 else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="one config only (default: the headline, config 3, followed by the secondary legs)")
    ap.add_argument("--scenarios", type=int, default=0, help="override S per GPU")
    ap.add_argument("--shard", choices=("scenarios", "rows"), default=None,
                    help="multi-GPU layout (SURVEY §8e): scenario sharding (default; 1m50k: rows)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--row-rounds", type=int, default=256,
                    help="pod-row sharding: rounds of the row-sharded multi-round loop to time (0: skip)")
    ap.add_argument("--no-kernel-events", action="store_true", default=os.environ.get("RSK_BENCH_NO_EVENTS") == "1",
                    help="time the steps without per-kernel HIP events")
    ap.add_argument("--pmc-json", default=PMC_JSON,
                    help="per-config PMC traffic (tools/pmc_summary.py, FETCH_SIZE x2-corrected)")
    ap.add_argument("--no-extra", action="store_true",
                    help="the headline line only (skip the secondary configs 2 / 4 / 5 of the default run)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU-only rehearsal of the multi-rank skeleton over gloo (no GPU, no librsk)")
    args = ap.parse_args()
    args.extra = args.config is None and not args.no_extra
    if args.config is None:
        args.config = "headline"
    args.steps_default = args.steps is None
    if args.steps is None:
        args.steps = 20
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    ablated = [k for k in ABLATION_VARS if os.environ.get(k, "0") not in ("", "0")]
    if ablated:
        sys.exit(f"[bench] refusing to run with wrong-result ablation switches set: {ablated}")

    # one process per GPU: without a launcher, --gpus N > 1 re-launches this
    # script as N ranks before anything here touches a GPU
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"[bench] WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}: "
                 "launch one rank per GPU with matching counts")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)

    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    args.rccl_world = dist.get_world_size() if world > 1 else 1

    cfg = dict(CONFIGS[args.config], key=args.config)
    if args.scenarios:
        cfg["S"] = args.scenarios
    line = run_config(args, cfg, world, rank, local, dev)
    # the secondary configs (BASELINE configs 2, 4 and 5, and config 5's per-rank
    # share at 8 GPUs), each with its own timing, parity and roofline, after the
    # headline's timed region and parity sample; the headline keys stay the
    # config-3 line's.  One GPU only: at N > 1 the line is the headline's alone.
    if args.extra and not args.scenarios and world == 1:
        line["configs"] = extra_configs(args, world, rank, local, dev)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


# Secondary legs of the default run: (block name, config, overrides).  Steps and
# warm-up are each config's own defaults (config 5: one call of R = 256 rounds).
EXTRA_LEGS = (
    ("config2", "2k64", {}),
    ("config4", "1m50k", {}),
    ("config5", "rounds", {}),
    ("config5_rank_share_8gpu", "rounds", {"S": 128}),
)


def extra_configs(args, world, rank, local, dev):
    """Run EXTRA_LEGS one after another in this process (inputs regenerated per
    leg, the previous leg's device memory released first) and return their
    lines by block name.  A leg that raises is recorded with its error and the
    others still run."""
    import copy
    import gc
    import traceback
    import torch
    out = {}
    for name, key, over in EXTRA_LEGS:
        a = copy.copy(args)
        a.steps, a.warmup, a.no_cpu_baseline, a.row_rounds = 20, 3, True, 256
        if key == "rounds":
            a.steps = 256
        cfg = dict(CONFIGS[key], key=key, **over)
        t0 = time.perf_counter()
        try:
            ln = run_config(a, cfg, world, rank, local, dev)
        except Exception as e:  # recorded, not fatal: the headline line still prints
            ln = {"error": f"{type(e).__name__}: {e}", "traceback": traceback.format_exc()[-2000:]}
        gc.collect()
        torch.cuda.empty_cache()
        if ln is not None:
            ln.pop("env", None)
            ln["leg_wall_s"] = round(time.perf_counter() - t0, 2)
            if "S" in over:
                ln["note"] = (f"config 5 at S = {over['S']} scenarios on one GPU: its per-rank share when the "
                              "1024 scenarios are sharded over 8 GPUs (DESIGN §6, what the split buys)")
            out[name] = ln
        log(f"[bench] leg {name}: {time.perf_counter() - t0:.1f}s")
    return out


def run_config(args, cfg, world, rank, local, dev):
    if cfg.get("rounds"):
        if args.steps_default:
            args.steps = 256   # config 5's R: one rsk_rounds_run call of 256 rounds
        return bench_rounds(args, cfg, world, rank, local, dev)
    return bench_car(args, cfg, world, rank, local, dev)


def bench_car(args, cfg, world, rank, local, dev):  # noqa: C901
    """One CAR config (headline, 2k64, 1m50k): the timed steps, the per-kernel
    breakdown, roofline, parity sample and, for config 4, the row-sharded rounds
    and kernel 3.  Returns rank 0's line (None on other ranks)."""
    import torch
    import torch.distributed as dist
    from rsk import _lib, api, synth
    from rsk import dist as rdist
    P, N, S = cfg["P"], cfg["N"], cfg["S"]
    by_rows = (args.shard or cfg.get("shard", "scenarios")) == "rows"
    t0 = time.time()
    if by_rows:  # pod-row sharding: full assign replica, a contiguous row range per rank
        c = synth.make_cluster(P, N, S=S, seed=0)
        rshard = rdist.row_shard_for(rank, world, c.row_ptr)
        my_rows, Q = rshard.rows, rshard.q
    else:        # scenario sharding: this rank's scenario range, every row
        shard = rdist.shard_for(rank, world, S)
        c = synth.make_cluster(P, N, S=S, seed=0, s0=shard.s0)
        my_rows, Q = None, P
    log(f"[bench] rank {rank}: generated {P}x{N}x{S} in {time.time() - t0:.1f}s")

    ctx = _lib.Context(local)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    t_plan = time.perf_counter()
    plan = api.CarPlan(c.row_ptr, c.col_idx, rows=my_rows, ctx=ctx)
    plan_ms = (time.perf_counter() - t_plan) * 1e3  # host C++ dedup + DFS order + tiling + upload, once per graph
    T = {k: torch.from_numpy(getattr(c, k)).to(dev) for k in ("assign", "cap_cpu", "use_cpu", "hazard")}
    out_t = torch.empty(max(Q, 1) * S, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)

    def step():
        plan.execute(T["assign"], S, T["cap_cpu"], T["use_cpu"], T["hazard"], N, out_t, None, device=True)

    names = ("car_direct", "car_prep", "car_tile", "car_side", "car_mid", "car_heavy")   # librsk's CAR timers

    def collect():
        out = {}
        for name in names:
            ms, n = ctx.kernel_time(name)
            if n:
                out[name] = {"avg_ms": ms / n, "launches": n, "per_step_ms": ms / args.steps}
        return out

    for _ in range(args.warmup):
        step()
    # per-kernel breakdown: an untimed pass with events around every launch
    ctx.reset_profiling()
    ctx.set_profiling(True)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    ctx.set_profiling(False)
    kernels = collect()
    # dominant kernel: the one carrying the most algorithmic bytes (car_tile at the
    # headline config); summed durations of launches that overlap on side streams
    # would not rank by time
    B = algorithmic_bytes(P, N, S, c.nnz)
    dom = max(kernels, key=lambda k: alg_bytes(k, P, N, S, plan.info(), B)) if kernels else None
    # the timed region: events only around the dominant kernel's launches —
    # unless the step is latency-bound (its launches under 50 us: config 2),
    # where an event pair costs as much as the kernel; then the steps are timed
    # bare and the kernel's duration is the breakdown pass's
    latency_bound = sum(v["per_step_ms"] for v in kernels.values()) < 0.05
    live_events = dom is not None and not args.no_kernel_events and not latency_bound
    ctx.reset_profiling()
    ctx.set_profile_only(dom)
    ctx.set_profiling(live_events)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    ctx.set_profiling(False)
    ctx.set_profile_only(None)
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    timed = collect()
    if dom in timed:  # the dominant kernel's duration measured inside the timed region
        kernels[dom] = dict(timed[dom], breakdown_pass_avg_ms=kernels[dom]["avg_ms"])
    elif dom is not None:
        kernels[dom]["duration_source"] = "breakdown pass (latency-bound step timed without events)"
    ms_step = elapsed * 1e3 / args.steps
    evals = P * N * S
    # scenario sharding: every rank scores P x N x S of its own (weak scaling);
    # row sharding: the ranks split one P x N x S batch (strong scaling)
    value = (1 if by_rows else world) * evals / (ms_step / 1e3)
    info = plan.info()
    gather_ms = None
    if by_rows and world > 1:  # the round's only data-path exchange, timed on its own
        torch.cuda.synchronize(dev)
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            full = rdist.gather_rows(out_t[: Q * S], rshard, S)
        torch.cuda.synchronize(dev)
        g = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        dist.all_reduce(g, op=dist.ReduceOp.MAX)
        gather_ms = float(g.item()) * 1e3 / args.steps
        del full

    # parity spot check against the oracle on sampled rows of this rank's batch
    from oracle import oracle as orc
    deg = np.diff(c.row_ptr)
    rng = np.random.default_rng(rank)
    r0 = rshard.r0 if by_rows else 0
    mine = deg[r0:r0 + Q]
    rows = np.unique(np.concatenate([np.argsort(mine)[-4:], rng.choice(Q, min(Q, 28), replace=False)]))
    rows = (rows + r0).astype(np.int32)
    got = out_t.view(Q, S)[torch.from_numpy(rows - r0).to(dev).long()].cpu().numpy().reshape(-1)
    exp, _ = orc.car(c.row_ptr, c.col_idx, c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, N, rows=rows,
                     threads=min(16, os.cpu_count() or 1))
    parity_ok = bool(np.array_equal(got, exp))

    rounds_leg = None
    if by_rows and args.row_rounds > 0:
        # the pod-row-sharded multi-round loop (rsk/dist.py RowShardedRounds): per
        # round an int64 all-reduce of the N*S CPU / mem partials, a MAX
        # all-reduce of the eviction key, the all-gather of changed slices and
        # the cut-cost all-reduce, around librsk's kernels on this rank's rows
        be = rdist.LibrskRoundsBackend(c.row_ptr, c.col_idx, c.pod_cpu, ctx=ctx, device=dev)
        rr = rdist.RowShardedRounds(rshard, be)
        a2 = T["assign"].clone()
        pc = torch.from_numpy(c.pod_cpu).to(dev)
        pm = torch.full((P,), 1 << 28, dtype=torch.int64, device=dev)   # synthetic 256 MiB per pod
        thr = 40   # the synthetic nodes run at 2-43 % CPU: only the hottest are hazards, so pods move
        rr.run(a2, T["use_cpu"], T["cap_cpu"], pc, pm, N, S, 1, threshold=thr)   # warm-up round
        a2.copy_(T["assign"])   # the timed rounds start from the generated state (use0 matches assign)
        a_start, u_start = T["assign"].cpu().numpy(), T["use_cpu"].cpu().numpy()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        res = rr.run(a2, T["use_cpu"], T["cap_cpu"], pc, pm, N, S, args.row_rounds, threshold=thr)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t1
        if world > 1:
            e = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
        R = args.row_rounds
        # parity of the whole loop (every scenario, every round) against
        # oracle_rounds from the same start: evictions, targets, the final
        # assign replica and usage, and the final cut count
        rows_parity = None
        if rank == 0:
            from oracle import oracle as orc
            t_par = time.perf_counter()
            ea, eu, eev, etg = orc.rounds(c.row_ptr, c.col_idx, c.pod_cpu, a_start, S, c.cap_cpu, u_start, N, R,
                                          threshold=thr, threads=cpu_threads()[0])
            ecut = orc.cut_cost(c.row_ptr, c.col_idx, ea, P, S)
            rows_parity = {
                "ok": bool(np.array_equal(res["evict"].cpu().numpy().reshape(-1), eev)
                           and np.array_equal(res["target"].cpu().numpy().reshape(-1), etg)
                           and np.array_equal(a2.cpu().numpy(), ea) and np.array_equal(res["use"].cpu().numpy(), eu)
                           and (R == 0 or np.array_equal(res["cut"][-1].cpu().numpy(), ecut))),
                "scope": f"all {S} scenarios x {R} rounds vs oracle_rounds (evictions, targets, final assign / use, "
                         f"final cut count)",
                "seconds": round(time.perf_counter() - t_par, 2)}
        # the same rounds with every librsk call, torch op and collective on the
        # current torch stream (no host sync between phases): the loop's rate
        a3 = T["assign"].clone()
        s2 = torch.cuda.Stream(dev)
        s2.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s2):
            be2 = rdist.LibrskRoundsBackend(c.row_ptr, c.col_idx, c.pod_cpu, device=dev, stream_ordered=True)
            rr2 = rdist.RowShardedRounds(rshard, be2)
            rr2.run(a3, T["use_cpu"], T["cap_cpu"], pc, pm, N, S, 1, threshold=thr)
            a3.copy_(T["assign"])
        def timed_run(nr):
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            t2 = time.perf_counter()
            with torch.cuda.stream(s2):
                out = rr2.run(a3, T["use_cpu"], T["cap_cpu"], pc, pm, N, S, nr, threshold=thr)
            torch.cuda.synchronize(dev)
            el2 = time.perf_counter() - t2
            if world > 1:
                e = torch.tensor([el2], dtype=torch.float64, device=dev)
                dist.all_reduce(e, op=dist.ReduceOp.MAX)
                el2 = float(e.item())
            return out, el2

        # the setup alone (R = 0: the rank's partials, the full cut count, the
        # u16 shadow, the final all-reduce), then the timed R rounds from the
        # generated state; steady state = (R rounds - setup) / R
        _, el0 = timed_run(0)
        a3.copy_(T["assign"])
        res2, el2 = timed_run(R)
        same = bool(torch.equal(res2["target"], res["target"]) and torch.equal(res2["cut"], res["cut"]))
        be2.close()
        rounds_leg = {"rounds": R, "threshold_pct": thr, "ms_per_round": round(el2 * 1e3 / R, 4),
                      "setup_ms": round(el0 * 1e3, 4),
                      "steady_ms_per_round": round((el2 - el0) * 1e3 / R, 4),
                      "stream_ordered_matches_synced": same,
                      "parity": rows_parity,
                      "ms_per_round_phase_synced": round(el * 1e3 / R, 4),
                      "phase_ms_per_round": {k: round(v / R, 4) for k, v in res["ms"].items()},
                      "scoring_only_ms_per_round": round(res["ms"]["place"] / R, 4),
                      "moves": int((res["target"] >= 0).sum().item()),
                      "collectives": "setup: int64 all-reduce of the N*S cpu partials; per round: int64 MAX "
                                     "all-reduce S, all-gather S changed slices, int64 all-reduce S cut cost; "
                                     "end: int64 all-reduce of the N*S cpu partials"}
        be.close()

    k3_leg = None
    if by_rows:
        # north-star kernel 3 over the whole batch (all P rows, device pointers):
        # per-node count / CPU / memory sums (rsk_node_reduce), the load std and the
        # cut cost, each its own launch timed with HIP events on the context's stream
        from rsk._lib import RSK_F_DEVICE, check
        pc = torch.from_numpy(c.pod_cpu).to(dev)
        pm = torch.from_numpy(c.pod_mem.astype(np.int64)).to(dev)
        cnt = torch.empty(N * S, dtype=torch.int32, device=dev)
        cs = torch.empty(N * S, dtype=torch.int64, device=dev)
        ms_ = torch.empty(N * S, dtype=torch.int64, device=dev)
        std = torch.empty(S, dtype=torch.float64, device=dev)
        cut = torch.empty(S, dtype=torch.int64, device=dev)
        rp_d = torch.from_numpy(c.row_ptr).to(dev)
        ci_d = torch.from_numpy(c.col_idx).to(dev)
        L, h = ctx.lib, ctx.handle

        def k3():
            check(L.rsk_node_reduce(h, T["assign"].data_ptr(), P, S, pc.data_ptr(), pm.data_ptr(), N, cnt.data_ptr(),
                                    cs.data_ptr(), ms_.data_ptr(), RSK_F_DEVICE))
            check(L.rsk_load_std(h, T["use_cpu"].data_ptr(), T["cap_cpu"].data_ptr(), N, S, std.data_ptr(),
                                 RSK_F_DEVICE))
            check(L.rsk_cut_cost(h, rp_d.data_ptr(), ci_d.data_ptr(), P, T["assign"].data_ptr(), S, None,
                                 cut.data_ptr(), RSK_F_DEVICE))
        k3()
        ctx.reset_profiling()
        ctx.set_profiling(True)
        reps = 10
        for _ in range(reps):
            k3()
        torch.cuda.synchronize(dev)
        ctx.set_profiling(False)
        k3_leg = {}
        alg3 = {"node_reduce": 4 * P * S + 12 * P + 20 * N * S, "load_std": 4 * N * S + 4 * N,
                "cut_cost": 4 * (P + 1) + 4 * c.nnz + 4 * P * S + 4 * c.nnz * S}
        try:
            with open(args.pmc_json) as f:
                pmc3 = json.load(f).get("kernel3", {}).get(cfg['key'], {})
        except (OSError, ValueError):
            pmc3 = {}
        for name in ("node_reduce", "load_std", "cut_cost"):
            tms, n = ctx.kernel_time(name)
            if n:
                k3_leg[name] = {"avg_ms": round(tms / n, 4), "launches_per_call": n // reps,
                                "algorithmic_bytes": alg3[name],
                                "algorithmic_GBps": round(alg3[name] / (tms / n / 1e3) / 1e9, 1)}
                e = pmc3.get(name)
                if e and e.get("S") == S:   # rocprof PMC bytes of the call's launches (tools/pmc_summary.py)
                    k3_leg[name]["traffic"] = e["hbm_bytes_per_call"]
                    k3_leg[name]["traffic_over_algorithmic"] = round(e["hbm_bytes_per_call"] / alg3[name], 3)
                    k3_leg[name]["traffic_source"] = e["source"]
        # parity of kernel 3 over the whole batch (every scenario): the oracle's
        # node sums and cut count exactly, its std within 1e-9 relative
        from oracle import oracle as orc
        a_h, u_h = T["assign"].cpu().numpy(), T["use_cpu"].cpu().numpy()   # the inputs k3() read
        ecnt, ecpu, emem = orc.node_reduce(a_h, P, S, c.pod_cpu, c.pod_mem.astype(np.int64), N)
        estd = orc.load_std(u_h, c.cap_cpu, N, S)
        ecut = orc.cut_cost(c.row_ptr, c.col_idx, a_h, P, S)
        k3_leg["parity_node_reduce_ok"] = bool(np.array_equal(cnt.cpu().numpy(), ecnt)
                                               and np.array_equal(cs.cpu().numpy(), ecpu)
                                               and np.array_equal(ms_.cpu().numpy(), emem))
        gstd = std.cpu().numpy()   # relative error; an all-equal batch (std 0) must match exactly
        k3_leg["parity_load_std_max_rel"] = float(np.max(np.where(estd == 0, np.where(gstd == 0, 0.0, np.inf),
                                                                  np.abs(gstd - estd) / np.where(estd == 0, 1, estd))))
        k3_leg["parity_cut_cost_ok"] = bool(np.array_equal(cut.cpu().numpy(), ecut))
        k3_leg["parity_sample_ok"] = bool(k3_leg["parity_node_reduce_ok"] and k3_leg["parity_cut_cost_ok"]
                                          and k3_leg["parity_load_std_max_rel"] <= 1e-9)
        k3_leg["parity_sample"] = f"all {S} scenarios of the batch: node_reduce / cut_cost exact, load_std 1e-9 rel"
        k3_leg["note"] = ("algorithmic bytes: node_reduce reads assign + pod cpu/mem and writes the N*S count/cpu/mem"
                          " words; load_std reads use and cap (its 20-B partials, one per (workgroup, scenario) after the in-LDS fold, not counted); cut_cost reads CSR + assign + one gather per edge")

    alg = {k: alg_bytes(k, P, N, S, info, B) for k in kernels}
    roof = None
    if dom in kernels and dom in alg:
        launches_per_step = kernels[dom]["launches"] / args.steps
        bytes_per_launch = alg[dom] / launches_per_step
        t = kernels[dom]["avg_ms"] / 1e3
        ach = bytes_per_launch / t / 1e9
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "algorithmic_bytes": int(bytes_per_launch)}
        try:
            with open(args.pmc_json) as f:
                pmc = json.load(f)
            entry = pmc.get("configs", {}).get(cfg['key'], {}).get(dom)
            if entry and entry.get("S") == S:
                roof["traffic"] = entry["hbm_bytes_per_launch"]
                roof["traffic_source"] = f"{os.path.relpath(args.pmc_json, REPO)} ({entry['source']})"
                roof["traffic_over_algorithmic"] = round(entry["hbm_bytes_per_launch"] / bytes_per_launch, 4)
                if entry.get("avg_us"):   # the same kernel's rocprofv3 kernel-trace average in the cited profile
                    roof["rocprof_avg_us"] = entry["avg_us"]
                    roof["frac_rocprof"] = round(bytes_per_launch / (entry["avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
                    roof["frac_note"] = ("frac: algorithmic bytes / this run's HIP-event average of the kernel inside "
                                         "the timed region; frac_rocprof: the same bytes / rocprof_avg_us, the "
                                         "rocprofv3 --kernel-trace --stats average in traffic_source (a builder run "
                                         "of the same library)")
        except (OSError, ValueError, KeyError):
            pass
    for k, v in kernels.items():
        if k in alg:
            v["algorithmic_GBps"] = round(alg[k] / (v["per_step_ms"] / 1e3) / 1e9, 1)
    step_ach = B / (ms_step / 1e3) / 1e9
    roof_step = {"bound": "hbm", "achieved": round(step_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(step_ach / HBM_PEAK_GBS, 4), "algorithmic_bytes": B,
                 "note": "whole CAR step (every launch of one execute, wall clock) vs SURVEY §8d B"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the cores this process may use (SURVEY §8d leg 3): the affinity mask
        # capped by the cgroup CPU quota, so no thread waits for CPU time
        threads, aff = cpu_threads()
        model, ncpu = cpu_model()
        # grow an evenly spaced pod sample until one timed pass takes >= 60 % of
        # --cpu-seconds (about 10-30 s of CPU work at the default)
        nrows = 64
        while True:
            sample = np.linspace(0, P - 1, nrows).astype(np.int32)
            t1 = time.perf_counter()
            orc.car(c.row_ptr, c.col_idx, c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, N, rows=sample,
                    threads=threads)
            dt = time.perf_counter() - t1
            if dt >= 0.6 * args.cpu_seconds or nrows >= P:
                break
            nrows = int(min(P, max(nrows + 1, nrows * args.cpu_seconds / max(dt, 1e-3))))
        cpu = {"value": round(nrows * S * N / dt, 1), "unit": "pod×node evals/s", "cores": threads, "kind": "port",
               "sample": f"{nrows} evenly spaced pods x {S} scenarios x {N} nodes ({dt:.1f}s), oracle/rsk_oracle.c "
                         f"literal CAR restatement, OpenMP {threads} threads",
               "seconds": round(dt, 2), "cpu_model": model, "host_logical_cpus": ncpu, "affinity_cpus": aff,
               "cgroup_cpu_quota": cgroup_cpu_quota(), "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
               "legs": python_legs(c, N, S)}

    line = None
    if rank == 0:
        line = {
            "metric": cfg["metric"], "value": round(value, 1), "unit": "pod×node evals/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong" if by_rows else "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
            "config": {"workload": cfg["name"], "pods": P, "nodes": N, "scenarios_per_gpu": S, "nnz": c.nnz,
                       "max_degree": int(deg.max()),
                       "parallelism": f"{'pod-row' if by_rows else 'scenario'}-sharded x{world}"},
            "roofline": roof, "roofline_step": roof_step, "cpu_baseline": cpu, "kernels": kernels,
            "parity_sample_ok": parity_ok, "hbm_bytes_algorithmic_per_step": B, "plan": info,
            "plan_create_ms": round(plan_ms, 1), "rccl_world": args.rccl_world, "env": rsk_env(),
        }
        if by_rows:
            line["rows_per_rank"] = Q
            line["roofline_scope"] = ("rank 0's rows: the plan's distinct neighbour pods of its row range "
                                      "(SURVEY §8e per-rank distinct-column roofline)")
            line["row_sharded_rounds"] = rounds_leg
            line["kernel3"] = k3_leg
            line["allgather_ms_per_step"] = None if gather_ms is None else round(gather_ms, 4)
            line["end_to_end_ms_per_step"] = round(ms_step + (gather_ms or 0.0), 4)
    plan.close()
    ctx.close()
    return line


if __name__ == "__main__":
    main()
