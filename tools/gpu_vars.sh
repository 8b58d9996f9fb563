#!/bin/bash
# Bench variants with split timers, no tests.
# usage: tools/gpu_vars.sh OUTDIR CONFIG[,CONFIG...] [VAR=val,VAR=val ...]
#   one bench per (config, variant); an empty variant "-" is the default build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/${1:-vars}
IFS=, read -ra cfgs <<< "${2:-headline}"
shift 2
mkdir -p "$out"
export TMPDIR=/tmp
[ $# -eq 0 ] && set -- -
for cfg in "${cfgs[@]}"; do
    for v in "$@"; do
        name="${cfg}_$(echo "$v" | tr ",=/" "___" | cut -c1-60)"
        envs=$( [ "$v" = - ] && echo "" || echo "$v" | tr "," " ")
        timeout -k 10 300 env RSK_TILE_TIMERS=1 RSK_SIDE_TIMERS=1 $envs python -u bench.py --config "$cfg" \
            --steps 20 --warmup 3 --no-cpu-baseline --row-rounds 0 > "$out/$name.log" 2>&1
        rc=$?
        echo "== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$out/$name.log" | head -1) $(grep -o '"parity_sample_ok": [a-z]*' "$out/$name.log")"
        [ $rc -ne 0 ] && { tail -15 "$out/$name.log"; exit $rc; }
        python3 - "$out/$name.log" <<'EOF'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print("   ", {k: round(v["per_step_ms"], 4) for k, v in d.get("kernels", {}).items()})
EOF
    done
done
