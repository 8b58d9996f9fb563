#!/bin/bash
# PMC calibration on the box: the available counters, then tools/membench/pmccal
# (known byte counts in the tile kernel's access widths) under separate PMC
# passes.  usage: tools/gpu_cal.sh OUTDIR ["CTR CTR" ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/cal}; shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$out/counters.txt" 2>&1 || echo "== list rc=$?"
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run -f csv -- tools/membench/pmccal > "$out/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$out/trace.log"; exit 1; }
k=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "$@"; do
  k=$((k+1))
  timeout -s KILL 60 rocprofv3 --pmc $set -d "$out/pmc$k" -o pmc -f csv -- tools/membench/pmccal > "$out/pmc$k.log" 2>&1
  rc=$?
  echo "== pass $k ($set) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$out/pmc$k.log"; exit $rc; }
done
exit 0
