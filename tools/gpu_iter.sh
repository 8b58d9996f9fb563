#!/bin/bash
# Iteration run: GPU parity suite, the headline bench with split timers, then
# one SQ counter pass (VALU / SALU / LDS / waves per kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/${1:-iter}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$out/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
for cfg in headline 1m50k; do
    RSK_HUB_TIMERS=1 RSK_TILE_TIMERS=1 timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --no-cpu-baseline > "$out/bench_$cfg.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$out/bench_$cfg.log"; exit $rc; }
    python3 - "$out/bench_$cfg.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print(sys.argv[1].split("/")[-1], d["ms_per_step"], d.get("parity_sample_ok"), {k: round(v["per_step_ms"], 4) for k, v in d["kernels"].items()})
PY
done
[ "${SQ:-1}" = 1 ] || exit 0
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d "$out/sq" -o p1 -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$out/sq_p1.log" 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -3 "$out/sq_p1.log"; exit $rc; }
python3 tools/sq_summary.py "$out/sq" | grep -v "^    SQ_\(WAVE_CYCLES\|BUSY_CYCLES\|INSTS_VMEM_WR\)" > "$out/sq_summary.txt"
grep -A6 "hub16\|mid16" "$out/sq_summary.txt"
