#!/bin/bash
# Round-2 evidence run: full -m gpu suite, drop-in latency, the headline bench
# with the CPU baseline, config 2 / 4 / 5 bench lines (profiles: gpu_r02_prof.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/${1:-r02final}
mkdir -p "$out"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    [ $rc -ne 0 ] && { tail -5 "$out/$name.log"; exit $rc; }
    return 0
}
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step dropin 300 python -u tools/dropin_latency.py --calls 40 --out "$out/dropin.json"
step bench_headline 400 python -u bench.py
step bench_2k64 200 python -u bench.py --config 2k64 --no-cpu-baseline
step bench_1m50k 300 python -u bench.py --config 1m50k --no-cpu-baseline
step bench_rounds 300 python -u bench.py --config rounds --no-cpu-baseline
