#!/bin/bash
# Tile-kernel ablations on the headline bench: full, no scoring, no image load, neither
# (RSK_ABLATE_TILE; results are wrong when ablated), side kernels serialized
# (RSK_OVERLAP=0), plus optional env variants: gpu_ablate.sh <outdir> [VAR=val,VAR2=val ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/ablate}; shift
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # run <name> [env...]
    local name=$1; shift
    env RSK_OVERLAP=0 "$@" timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$out/$name.log") $(python3 -c '
import json,sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d=json.loads(l); print({k: round(v["per_step_ms"],3) for k,v in d["kernels"].items()}, d["parity_sample_ok"])' "$out/$name.log")"
    [ $rc -ne 0 ] && { tail -5 "$out/$name.log"; exit $rc; }
    return 0
}
run full
run noscore RSK_ABLATE_TILE=2
run noload RSK_ABLATE_TILE=1
run neither RSK_ABLATE_TILE=3
for v in "$@"; do run "$(echo "$v" | tr ",=/" "___" | cut -c1-60)" $(echo "$v" | tr "," " "); done
