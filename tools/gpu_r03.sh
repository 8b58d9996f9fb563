#!/bin/bash
# Round-3 iteration: CAR parity (default plan, then 17..32 rows on the side
# kernel), then headline / config-4 bench variants with split timers.
# usage: tools/gpu_r03.sh OUTDIR [test|notest] [VAR=val,VAR=val ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/${1:-r03}
mode=${2:-test}
shift 2
mkdir -p "$out"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T) $(grep -o '"ms_per_step": [0-9.]*' "$out/$name.log" | head -1) $(grep -o '"parity_sample_ok": [a-z]*' "$out/$name.log")"
    [ $rc -ne 0 ] && { tail -15 "$out/$name.log"; exit $rc; }
    return 0
}
if [ "$mode" = test ]; then
    [ -n "$SKIP_BASE_TEST" ] || step pytest_car 500 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread
    [ -n "$SKIP_L16_TEST" ] || step pytest_car_l16 400 env RSK_LIGHT_MAX=16 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -v -k "car" --timeout 200 --timeout-method thread
fi
bench() {  # bench <name> <config> [env...]
    local name=$1 cfg=$2; shift 2
    step "bench_$name" 300 env RSK_TILE_TIMERS=1 RSK_SIDE_TIMERS=1 "$@" python -u bench.py --config "$cfg" --steps 20 --warmup 3 --no-cpu-baseline
    python3 - "$out/bench_$name.log" <<'EOF'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print("   ", {k: round(v["per_step_ms"], 4) for k, v in d.get("kernels", {}).items()})
EOF
}
bench head headline
bench head_l16 headline RSK_LIGHT_MAX=16
bench 1m50k 1m50k
bench 1m50k_l16 1m50k RSK_LIGHT_MAX=16
for v in "$@"; do bench "v_$(echo "$v" | tr ",=/" "___" | cut -c1-60)" headline $(echo "$v" | tr "," " "); done
if [ -n "$DROPIN" ]; then
    step dropin 300 python -u tools/dropin_latency.py --calls 40 --out "$out/dropin.json"
    grep -o '"config.*' "$out/dropin.log" | cut -c1-200
fi
