#!/bin/bash
# Headline bench under env variants (default settings otherwise):
#   gpu_sweep.sh <outdir> [--config C] "" "VAR=val,VAR2=val" ...
# ("" = defaults).  Prints ms_per_step, per-kernel ms and the parity flag per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/sweep}; shift
cfg=headline
if [ "$1" = "--config" ]; then cfg=$2; shift 2; fi
mkdir -p "$out"
export TMPDIR=/tmp
for v in "$@"; do
    name=$(echo "${v:-default}" | tr ",=/" "___" | cut -c1-60)
    env $(echo "$v" | tr "," " ") timeout -k 10 200 python -u bench.py --config "$cfg" --steps 20 --warmup 3 \
        --no-cpu-baseline > "$out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$out/$name.log") $(python3 -c '
import json,sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d=json.loads(l); print({k: round(v["per_step_ms"],3) for k,v in d["kernels"].items()}, d["parity_sample_ok"])' "$out/$name.log")"
    [ $rc -ne 0 ] && { tail -5 "$out/$name.log"; exit $rc; }
done
exit 0
