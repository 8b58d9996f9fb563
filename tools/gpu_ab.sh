#!/bin/bash
# Interleaved A/B of env variants on the headline bench (noise control).
# usage: gpu_ab.sh REPS VAR=v[,VAR2=v] ...   ("base" = no extra env)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
reps=$1; shift
for r in $(seq 1 "$reps"); do
    k=0
    for v in "$@"; do
        k=$((k + 1))
        name=v$k
        envs=$(echo "$v" | tr "," " "); [ "$v" = base ] && envs=""
        env $envs timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/$name.$r.log 2>&1
        rc=$?
        echo "$r $name [$(echo "$v" | sed 's#.*/##' | cut -c1-60)] rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$name.$r.log) $(grep -o '"car_tile": {"avg_ms": [0-9.]*' gpurun_out/ab/$name.$r.log | cut -c24-30) $(grep -o '"parity_sample_ok": [a-z]*' gpurun_out/ab/$name.$r.log)"
        [ $rc -ne 0 ] && { tail -5 gpurun_out/ab/$name.$r.log; exit $rc; }
    done
done
exit 0
