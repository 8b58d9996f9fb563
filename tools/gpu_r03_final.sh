#!/bin/bash
# Round-3 evidence on one box: the default bench line of every config, the
# drop-in latency, then rocprof kernel-trace stats + PMC passes (headline, 1m50k, 2k64).
# usage: tools/gpu_r03_final.sh OUTDIR [noprof]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/${1:-r03final}
mkdir -p "$out"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T) $(grep -o '"ms_per_step": [0-9.]*' "$out/$name.log" | head -1) $(grep -o '"parity_sample_ok": [a-z]*' "$out/$name.log")"
    [ $rc -ne 0 ] && { tail -15 "$out/$name.log"; exit $rc; }
    return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_headline 600 python -u bench.py
step bench_2k64 300 python -u bench.py --config 2k64 --no-cpu-baseline
step bench_1m50k 600 python -u bench.py --config 1m50k --no-cpu-baseline
step bench_rounds 300 python -u bench.py --config rounds --no-cpu-baseline
step dropin 400 python -u tools/dropin_latency.py --calls 40 --out "$out/dropin.json"
[ "$2" = noprof ] && exit 0
for c in headline 1m50k 2k64; do
    ./tools/gpu_prof.sh $c "$out/prof_$c" > "$out/prof_$c.log" 2>&1 || { tail -5 "$out/prof_$c.log"; exit 1; }
    echo "== prof $c done $(date +%T)"
done
