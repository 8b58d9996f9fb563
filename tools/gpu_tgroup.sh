#!/bin/bash
# Tile-group A/B on the headline: per value, the bench (no CPU baseline) and a
# FETCH_SIZE pass.  usage: tools/gpu_tgroup.sh OUTDIR G...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/tg}; shift
mkdir -p "$out"
export TMPDIR=/tmp RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_knobs.so
for g in "$@"; do
  export RSK_TILE_GROUP=$g
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > "$out/bench_g$g.log" 2>&1 || { echo "bench g$g failed"; tail -5 "$out/bench_g$g.log"; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d "$out/pmc_g$g" -o fetch -f csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$out/pmc_g$g.log" 2>&1 || { echo "pmc g$g failed"; exit 1; }
  echo "== g$g $(grep -o '"ms_per_step": [0-9.]*' "$out/bench_g$g.log")"
done
exit 0
