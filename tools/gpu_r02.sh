#!/bin/bash
# Round-2 GPU check: bounds-checked library on the CAR parity tests, then the
# product library on every -m gpu test, then the headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/${1:-r02}
mkdir -p "$out"
export TMPDIR=/tmp
RSK_LIB=$PWD/kubernetes-rescheduling_amd/rsk/librsk_dbg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "car" > "$out/pytest_dbg.log" 2>&1
rc=$?; tail -3 "$out/pytest_dbg.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$out/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$out/bench.log" 2>&1
rc=$?; tail -c 1500 "$out/bench.log"; exit $rc
