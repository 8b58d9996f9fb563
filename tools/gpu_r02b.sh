#!/bin/bash
# Round-2 re-check: GPU parity suite, then per-kernel breakdowns (split tile and
# hub timers) at configs 3 and 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/${1:-r02b}
mkdir -p "$out"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T) $(grep -o '"ms_per_step": [0-9.]*' "$out/$name.log")"
    [ $rc -ne 0 ] && { tail -5 "$out/$name.log"; exit $rc; }
    return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_headline 300 python -u bench.py --steps 20 --no-cpu-baseline
step split_headline 300 env RSK_TILE_TIMERS=1 RSK_HUB_TIMERS=1 python -u bench.py --steps 20 --no-cpu-baseline
step split_1m50k 300 env RSK_TILE_TIMERS=1 RSK_HUB_TIMERS=1 python -u bench.py --config 1m50k --steps 20 --no-cpu-baseline
for f in "$out"/split_*.log; do
    python3 - "$f" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print(sys.argv[1].split("/")[-1], d["ms_per_step"], {k: round(v["per_step_ms"], 4) for k, v in d["kernels"].items()})
PY
done
