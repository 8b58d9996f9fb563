#!/bin/bash
# Quick GPU iteration: parity tests, then the headline bench (+ optional env variants).
# usage: gpu_quick.sh [test|notest] [VAR=val ...]   (each VAR=val runs one extra bench variant)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/q
export TMPDIR=/tmp
if [ "${1:-test}" = test ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q/pytest_gpu.log 2>&1
    rc=$?; tail -4 gpurun_out/q/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
shift
bench() {  # bench <name> [env...]
    local name=$1; shift
    env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/q/bench_$name.log 2>&1
    local rc=$?
    echo "== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/q/bench_$name.log) $(grep -o '"kernels": {.*}}, "parity' gpurun_out/q/bench_$name.log | python3 -c 'import sys,json; s=sys.stdin.read().strip(); d=json.loads(s[11:-9]) if s else {}; print({k: round(v["per_step_ms"],3) for k,v in d.items()})')"
    grep -o '"parity_sample_ok": [a-z]*' gpurun_out/q/bench_$name.log
    [ $rc -ne 0 ] && { tail -5 gpurun_out/q/bench_$name.log; exit $rc; }
    return 0
}
bench base
for v in "$@"; do bench "$(echo "$v" | tr "/" "_" | cut -c1-80)" $(echo "$v" | tr "," " "); done
