#!/bin/bash
# One GPU session: parity tests, smoke, a short bench, and a rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash / timeout (rc >= 2) stops the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step pytest_gpu 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
    step smoke 180 python -u __graft_entry__.py smoke
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 400 python -u bench.py --steps 20 --warmup 3
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    step rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
    # one counter group per pass (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2: never together)
    step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o fetch -f csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
    step pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc -o write -f csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
    step pmc_l2 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc -o l2 -f csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
fi
if [ "$MODE" = ablate ]; then
    step bench_full 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline
    RSK_ABLATE_TILE=2 step bench_noscore 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline
    RSK_ABLATE_TILE=1 step bench_noload 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline
    RSK_ABLATE_TILE=3 step bench_nothing 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline
fi
