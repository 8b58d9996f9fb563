#!/bin/bash
# SQ / TA counter passes on the headline bench, or on SQ_CMD (one rocprofv3 --pmc run per group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/sq gpurun_out/sq_abl "${SQ_OUT:-gpurun_out/sq}"
export TMPDIR=/tmp RSK_OVERLAP=0
OUT=${SQ_OUT:-gpurun_out/sq}
B=${SQ_CMD:-"python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"}
pass() {  # pass <name> <counters...>
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT -o "$name" -f csv -- $B > "$OUT/$name.log" 2>&1
    local rc=$?; echo "== $name rc=$rc"; [ $rc -ne 0 ] && { tail -3 "$OUT/$name.log"; exit $rc; }
    return 0
}
pass p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass p2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM
pass p3 TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ TCP_TCC_WRITE_REQ
