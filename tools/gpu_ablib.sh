#!/bin/bash
# A/B of two librsk builds on one box: the product librsk.so against
# rsk/librsk_$VAR.so (RSK_LIB), benches interleaved.  usage:
#   tools/gpu_ablib.sh OUTDIR VAR "pytest -k expression" config [config...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/${1:-ablib}; var=$2; kexpr=$3; shift 3
mkdir -p "$out"
export TMPDIR=/tmp
alt=kubernetes-rescheduling_amd/rsk/librsk_$var.so
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$out/$name.log" | head -1) $(grep -o '"parity_sample_ok": [a-z]*' "$out/$name.log" | head -1) $(grep -E -o '[0-9]+ (passed|failed)[^=]*' "$out/$name.log" | tail -1)"
    [ $rc -ne 0 ] && { tail -20 "$out/$name.log"; exit $rc; }
    return 0
}
if [ -n "$kexpr" ]; then
    run "pytest_$var" 600 env RSK_LIB=$alt python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$kexpr"
fi
for rep in 1 2; do
    for cfg in "$@"; do
        run "b_${cfg}_base_$rep" 300 python -u bench.py --config "$cfg" --no-cpu-baseline --row-rounds 0
        run "b_${cfg}_${var}_$rep" 300 env RSK_LIB=$alt python -u bench.py --config "$cfg" --no-cpu-baseline --row-rounds 0
    done
done
exit 0
