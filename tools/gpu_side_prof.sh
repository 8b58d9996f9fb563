#!/bin/bash
# Side-kernel counters on the headline bench: kernel trace + SQ passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${SQ_OUT:-gpurun_out/sideprof}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $OUT -o trace -f csv -- $B > "$OUT/trace.log" 2>&1 || { echo trace failed; tail -3 "$OUT/trace.log"; exit 1; }
echo "== trace ok"
pass() {  # pass <name> <counters...>
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT -o "$name" -f csv -- $B > "$OUT/$name.log" 2>&1
    local rc=$?; echo "== $name rc=$rc"; [ $rc -ne 0 ] && { tail -3 "$OUT/$name.log"; exit $rc; }
    return 0
}
pass p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass p2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM
python3 tools/sq_summary.py $OUT
