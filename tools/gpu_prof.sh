#!/bin/bash
# Profile one bench config: rocprofv3 kernel trace + stats, then separate PMC
# passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss: never two TCC-heavy counters in
# one pass).  usage: gpu_prof.sh <config> <outdir> [extra bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
cfg=${1:-headline}; out=${2:-gpurun_out/prof_$cfg}; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
B="python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline $*"
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -s KILL "$secs" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    [ $rc -ne 0 ] && { tail -5 "$out/$name.log"; exit $rc; }
    return 0
}
step trace 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -f csv -- $B
step fetch 180 rocprofv3 --pmc FETCH_SIZE -d "$out/pmc" -o fetch -f csv -- $B
step write 180 rocprofv3 --pmc WRITE_SIZE -d "$out/pmc" -o write -f csv -- $B
step l2 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$out/pmc" -o l2 -f csv -- $B
grep -h '"ms_per_step"' "$out/trace.log" | cut -c1-300
