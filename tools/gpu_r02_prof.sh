#!/bin/bash
# rocprof profiles (trace + FETCH/WRITE/L2 passes) of configs headline, 2k64, 1m50k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/${1:-r02prof}
mkdir -p "$out"
for c in headline 2k64 1m50k; do
    ./tools/gpu_prof.sh $c "$out/prof_$c" > "$out/prof_$c.log" 2>&1 || { tail -5 "$out/prof_$c.log"; exit 1; }
    echo "== prof $c done $(date +%T)"
done
