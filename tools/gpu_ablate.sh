#!/bin/bash
# Tile-kernel ablations + SQ counters (one GPU session).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/abl/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    grep -o '"car_tile": {[^}]*}' "gpurun_out/abl/$name.log" | head -1
    if [ $rc -ne 0 ]; then tail -5 "gpurun_out/abl/$name.log"; exit $rc; fi
}
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline"
run full 200 $B
RSK_ABLATE_TILE=1 run noload 200 $B
RSK_ABLATE_TILE=2 run noscore 200 $B
RSK_ABLATE_TILE=3 run nothing 200 $B
RSK_TILE_SL=16 run sl16 200 $B
RSK_TILE_SL=64 run sl64 200 $B
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/abl/avail.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/abl/pmc -o sq -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abl/pmc_sq.log 2>&1
echo "pmc rc=$?"
