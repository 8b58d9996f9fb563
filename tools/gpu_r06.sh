#!/bin/bash
# GPU session on one box.  usage: tools/gpu_r06.sh OUTDIR [steps...]
# steps: test (pytest -m gpu), smoke, bench (headline), b2k (config 2),
#        b1m (config 4), brounds (config 5), prof (rocprof trace + PMC of headline
#        and 1m50k), profh / prof1m (one config), dropin, nrb (tools/nrbench.py),
#        nrprof (its kernel trace), pmc:LIB:CONFIG:ENV (FETCH / WRITE passes of tools/tilebench.py
#        with librsk_LIB.so — base: the product — and ENV=a=1,b=2 or -)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/${1:-r06}; shift
mkdir -p "$out"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T) $(grep -o '"ms_per_step": [0-9.]*' "$out/$name.log" | head -1) $(grep -o '"parity_sample_ok": [a-z]*' "$out/$name.log" | head -1) $(grep -E -o '[0-9]+ (passed|failed)[^=]*' "$out/$name.log" | tail -1)"
    [ $rc -ne 0 ] && { tail -25 "$out/$name.log"; exit $rc; }
    return 0
}
for s in "${@:-test smoke bench}"; do
  for w in $s; do
    case $w in
      test) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
      test:*) step "pytest_${w#test:}" 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${w#test:}" ;;
      smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
      bench) step bench_headline 600 python -u bench.py ;;
      b2k) step bench_2k64 300 python -u bench.py --config 2k64 --no-cpu-baseline ;;
      b1m) step bench_1m50k 600 python -u bench.py --config 1m50k --no-cpu-baseline ;;
      brounds) step bench_rounds 300 python -u bench.py --config rounds --no-cpu-baseline ;;
      ab:*) kv=${w#ab:}; step "ab_${kv//[=,]/_}" 300 env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_knobs.so ${kv//,/ } python -u bench.py --no-cpu-baseline ;;
      abr:*) kv=${w#abr:}; step "abr_${kv//[=,]/_}" 300 env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_knobs.so ${kv//,/ } python -u bench.py --config rounds --no-cpu-baseline ;;
      sb:*) kv=${w#sb:}; step "sb_${kv//[=,]/_}" 300 env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_abl.so ${kv//,/ } python -u tools/sidebench.py ;;
      hp:*) step "hostprobe_${w#hp:}" 300 python -u tools/hostprobe.py "${w#hp:}" ;;
      rprof) step rounds_prof 300 env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_rprof.so python -u bench.py --config rounds --no-cpu-baseline --no-kernel-events ;;
      rprof128) step rounds_prof128 300 env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_rprof.so python -u bench.py --config rounds --scenarios 128 --no-cpu-baseline --no-kernel-events ;;
      pmc:*) v=${w#pmc:}; lib=${v%%:*}; v=${v#*:}; cfg=${v%%:*}; kv=${v#*:}; [ "$kv" = "-" ] && kv=""
             tag="${lib}_${cfg}_${kv//[=,]/_}"; envs=${kv//,/ }
             [ "$lib" != base ] && envs="RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_$lib.so $envs"
             for c in FETCH_SIZE WRITE_SIZE; do
               step "pmc_${tag}_$c" 240 env $envs rocprofv3 --pmc $c -d "$out/pmc_$tag/$c" -o p -f csv -- python3 tools/tilebench.py --config $cfg --steps 10
             done
             python3 tools/pmc_quick.py "$out/pmc_$tag" | tee "$out/pmc_${tag}_summary.txt" ;;
      ab1m:*) lib=${w#ab1m:}; for rep in 1 2; do
               step "ab1m_base_$rep" 300 python -u bench.py --config 1m50k --no-cpu-baseline
               step "ab1m_${lib}_$rep" 300 env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_$lib.so python -u bench.py --config 1m50k --no-cpu-baseline
             done ;;
      abh:*) lib=${w#abh:}; for rep in 1 2; do
               step "abh_base_$rep" 300 python -u bench.py --config headline --no-cpu-baseline
               step "abh_${lib}_$rep" 300 env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_$lib.so python -u bench.py --config headline --no-cpu-baseline
             done ;;
      prof1m:*) lib=${w#prof1m:}; env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_$lib.so ./tools/gpu_prof.sh 1m50k "$out/prof_1m50k_$lib" > "$out/prof_1m50k_$lib.log" 2>&1 || { tail -5 "$out/prof_1m50k_$lib.log"; exit 1; }
                echo "== prof1m $lib done $(date +%T)" ;;
      tnr:*) lib=${w#tnr:}; step "pytest_nr_$lib" 300 env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_$lib.so python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "node_reduce or kernel3 or write_guard" ;;
      bnoev) step bench_noevents 600 python -u bench.py --no-cpu-baseline --no-kernel-events ;;
      nr:*) kv=${w#nr:}; step "nr_${kv//[=,]/_}" 300 env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_abl.so ${kv//,/ } python -u tools/nrbench.py ;;
      nrk:*) kv=${w#nrk:}; step "nrk_${kv//[=,]/_}" 300 env RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_knobs.so ${kv//,/ } python -u tools/nrbench.py ;;
      nrprof:*) lib=${w#nrprof:}; envs=""; [ "$lib" != base ] && envs="RSK_LIB=kubernetes-rescheduling_amd/rsk/librsk_$lib.so"
                env $envs ./tools/gpu_nrprof.sh "$out/nrprof_${lib}_$RANDOM" > "$out/nrprof_$lib.log" 2>&1 || { tail -5 "$out/nrprof_$lib.log"; exit 1; }
                cat "$out/nrprof_$lib.log" ;;
      nrb) step nrbench 300 python -u tools/nrbench.py ;;
      nrprof) ./tools/gpu_nrprof.sh "$out/nrprof" > "$out/nrprof.log" 2>&1 || { tail -5 "$out/nrprof.log"; exit 1; }; cat "$out/nrprof.log" ;;
      dropin) step dropin 400 python -u tools/dropin_latency.py --calls 40 --out "$out/dropin.json" ;;
      prof) for c in headline 1m50k; do
              ./tools/gpu_prof.sh $c "$out/prof_$c" > "$out/prof_$c.log" 2>&1 || { tail -5 "$out/prof_$c.log"; exit 1; }
              echo "== prof $c done $(date +%T)"; done ;;
      profh) ./tools/gpu_prof.sh headline "$out/prof_headline" > "$out/prof_headline.log" 2>&1 || { tail -5 "$out/prof_headline.log"; exit 1; } ;;
      prof1m) ./tools/gpu_prof.sh 1m50k "$out/prof_1m50k" > "$out/prof_1m50k.log" 2>&1 || { tail -5 "$out/prof_1m50k.log"; exit 1; } ;;
      *) echo "unknown step $w"; exit 2 ;;
    esac
  done
done
