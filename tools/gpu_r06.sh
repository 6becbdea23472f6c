#!/bin/bash
# Round-6 GPU call (one gpurun): the steps named on the command line, each under
# its own time limit; a failing step ends the call (test failures, pytest rc 1,
# excepted: the GPU is fine then and later steps still run).
#   tools/gpu_r06.sh [tests] [bench] [cq-<var>] [q-<var>] [c5q-<var>] [e8q-<var>] [iq-<var>] ...
# <var> = base (the in-tree libmtsg.so) or a Makefile VARIANTS name (my-mitsuba_amd/var/).
O=gpurun_out/r6
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 3 "$O/$name.log" | cut -c1-2500; if [ $rc -ne 0 ] && ! { [ "${name%%-*}" = tests ] && [ $rc -eq 1 ]; }; then exit $rc; fi; }
lib() { local v=${1%@*}; if [ "$v" = base ]; then echo ""; else echo "my-mitsuba_amd/var/libmtsg_$v.so"; fi; }
PYT="python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread"
Q="--no-cpu --no-parity"
for w in ${*:-tests bench}; do
  case $w in
    tests) step tests 900 $PYT tests ;;
    tfar-*) v=${w#tfar-}; MTSG_LIB=$(lib $v) step $w 300 $PYT tests/test_gpu_instancing.py -k far_away ;;
    tests-parity) step tests-parity 600 $PYT tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_c4.py ;;
    tests-inst) step tests-inst 600 $PYT tests/test_gpu_instancing.py tests/test_gpu_edge_rays.py tests/test_gpu_finish.py ;;
    vtests-*) v=${w#vtests-}; MTSG_LIB=$(lib $v) step $w 900 $PYT tests ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 3 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    # C3 with the instrumented pass (SIMD efficiency, iterations) / without it
    cq-*) v=${w#cq-}; MTSG_LIB=$(lib $v) step $w 300 python bench.py --steps 10 --warmup 3 $Q ;;
    q-*) v=${w#q-}; MTSG_LIB=$(lib $v) step $w 300 python bench.py --steps 10 --warmup 3 $Q --no-count ;;
    iq-*) v=${w#iq-}; MTSG_LIB=$(lib $v) step $w 300 python bench.py --steps 5 --warmup 2 --instancing two-level $Q ;;
    c5q-*) v=${w#c5q-}; MTSG_LIB=$(lib $v) step $w 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 $Q --no-count ;;
    # the shading event sort A/B, both in append order
    ssq-*) v=${w#ssq-}; MTSG_LIB=$(lib $v) step $w 300 python bench.py --steps 10 --warmup 3 $Q --no-count --ray-order 0 ;;
    ssc5-*) v=${w#ssc5-}; MTSG_LIB=$(lib $v) step $w 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 $Q --no-count --ray-order 0 ;;
    ssc2-*) v=${w#ssc2-}; MTSG_LIB=$(lib $v) step $w 300 python bench.py --steps 5 --warmup 2 --workload cbox $Q --no-count --ray-order 0 ;;
    qro0) step qro0 300 python bench.py --steps 10 --warmup 3 $Q --ray-order 0 ;;
    c5ro0) step c5ro0 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 $Q --no-count --ray-order 0 ;;
    e8bands*) step $w 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 $Q --no-count --share-layout bands --balance-rounds 6 ;;
    e8spread*) step $w 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 $Q --no-count --balance-rounds 6 ;;
    e8ro0) step e8ro0 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 $Q --no-count --ray-order 0 ;;
    ktro0) step ktro0 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_ro0 -o kt -- python3 bench.py --pmc-pass $Q --no-count --steps 1 --warmup 1 --ray-order 0 ;;
    c5g) step c5g 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 $Q --no-count --shade-generic ;;
    # kd-tree build properties (bench.py --kd-props), e.g. kdq:kdIntersectionCost=10,kdStopPrims=3
    # tail-kernel switch point (paths; bench.py --finish-paths): c5f-<N> / qf-<N> / e8f-<N>
    c5f-*) n=${w#c5f-}; step $w 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 $Q --no-count --finish-paths ${n%@*} ;;
    qf-*) n=${w#qf-}; step $w 300 python bench.py --steps 10 --warmup 3 $Q --no-count --finish-paths ${n%@*} ;;
    e8f-*) n=${w#e8f-}; step $w 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 $Q --no-count --finish-paths ${n%@*} ;;
    # batches in flight (C5): c5l:<lanes>:<stagger>:<batch paths>
    c5l:*) IFS=: read -r _ ln sg bp <<< "$w"; step "c5l-$ln-$sg-$bp" 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 $Q --no-count --lanes $ln --stagger $sg --batch-paths $bp ;;
    # batch size (paths; bench.py --batch-paths): c5b-<N>
    c5b-*) n=${w#c5b-}; step $w 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 $Q --no-count --batch-paths ${n%@*} ;;
    # tail kernel's shading threshold (bench.py --finish-shade-min): c5sm-<n> / e8sm-<n>
    c5sm-*) n=${w#c5sm-}; step $w 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 $Q --no-count --finish-shade-min ${n%@*} ;;
    qsm-*) n=${w#qsm-}; step $w 300 python bench.py --steps 10 --warmup 3 $Q --no-count --finish-shade-min ${n%@*} ;;
    iqsm-*) n=${w#iqsm-}; step $w 300 python bench.py --steps 5 --warmup 2 --instancing two-level $Q --no-count --finish-shade-min ${n%@*} ;;
    e8sm-*) n=${w#e8sm-}; step $w 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 $Q --no-count --finish-shade-min ${n%@*} ;;
    kdq:*) p=${w#kdq:}; step "kdq-${p//[=,]/_}" 300 python bench.py --steps 10 --warmup 3 $Q --no-count --kd-props "$p" ;;
    kdi:*) p=${w#kdi:}; step "kdi-${p//[=,]/_}" 300 python bench.py --steps 5 --warmup 2 --instancing two-level $Q --no-count --kd-props "$p" ;;
    kdc5:*) p=${w#kdc5:}; step "kdc5-${p//[=,]/_}" 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 $Q --no-count --kd-props "$p" ;;
    qg) step qg 300 python bench.py --steps 10 --warmup 3 $Q --no-count --shade-generic ;;
    c2q-*) v=${w#c2q-}; MTSG_LIB=$(lib $v) step $w 300 python bench.py --steps 5 --warmup 2 --workload cbox $Q --no-count ;;
    e8q-*) v=${w#e8q-}; MTSG_LIB=$(lib $v) step $w 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 $Q --no-count ;;
    ranks)
      # the launcher path (as the driver runs it) and the self-launching path,
      # two ranks on this one GPU; then the refusal without --allow-shared
      step ranks-torchrun 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --allow-shared
      step ranks-self 600 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --allow-shared
      echo "== ranks-refuse"; timeout -k 10 300 python bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu > $O/ranks-refuse.log 2>&1; echo "ranks-refuse rc=$? (non-zero expected)"; tail -n 2 $O/ranks-refuse.log ;;
    c5) step c5 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 ;;
    c2) step c2 600 python bench.py --steps 5 --warmup 2 --workload cbox ;;
    inst) step inst 300 python bench.py --steps 5 --warmup 2 --instancing two-level --no-cpu --no-parity ;;
    e8) step e8 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 --no-cpu --no-parity ;;
    stats-c3) step stats-c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-parity --no-count ;;
    stats-c5) step stats-c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 bench.py --steps 2 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 --no-cpu --no-parity --no-count ;;
    # per-launch kernel durations of one frame (tools/launch_times.py)
    kt-*) v=${w#kt-}; MTSG_LIB=$(lib $v) step $w 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 bench.py --pmc-pass $Q --no-count --steps 1 --warmup 1 ;;
    kte8-*) v=${w#kte8-}; MTSG_LIB=$(lib $v) step $w 300 rocprofv3 --kernel-trace --output-format csv -d $O/kte8_$v -o kt -- python3 bench.py --pmc-pass --emulate-ranks 8 $Q --no-count --steps 1 --warmup 1 ;;
    ktc5-*) v=${w#ktc5-}; MTSG_LIB=$(lib $v) step $w 300 rocprofv3 --kernel-trace --output-format csv -d $O/ktc5_$v -o kt -- python3 bench.py --pmc-pass --workload c5 --width 1920 --height 1080 --spp 1024 $Q --no-count --steps 1 --warmup 0 ;;
    kti-*) v=${w#kti-}; MTSG_LIB=$(lib $v) step $w 300 rocprofv3 --kernel-trace --output-format csv -d $O/kti_$v -o kt -- python3 bench.py --pmc-pass --instancing two-level $Q --no-count --steps 1 --warmup 1 ;;
    # FETCH_SIZE against known bytes for streams and gathers (tools/fetch_calib.hip)
    calib) step calib 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/calib -o calib -- tools/fetch_calib ;;
    # TCC hit rate / traffic of the ray orders (profiles/r06_ray_order.txt; sets not quoted by bench)
    pmcro-base) bash tools/gpu_pmc_config.sh r06ro append --ray-order 0 || exit $? ;;
    pmcro-sorted) bash tools/gpu_pmc_config.sh r06ro sorted --ray-order 1 || exit $? ;;
    pmcro-shuf1) MTSG_LIB=$(lib shuf1) bash tools/gpu_pmc_config.sh r06ro shuf1 || exit $? ;;
    # SQ counters per kernel (tools/sq_by_kernel.py): sq-c3 / sq-c5, one frame per pass (C5 at 256 spp)
    sq-c3|sq-c5|sq-inst)
      t=${w#sq-}; A="--pmc-pass $Q --no-count --steps 1 --warmup 0"
      [ $t = c5 ] && A="$A --workload c5 --width 1920 --height 1080 --spp 256"
      [ $t = inst ] && A="$A --instancing two-level"
      D=$O/sq_$t; mkdir -p $D
      step sq-$t-p1 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $D -o p1 -- python3 bench.py $A
      step sq-$t-p2 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $D -o p2 -- python3 bench.py $A
      python3 tools/sq_by_kernel.py $D/p1_counter_collection.csv $D/p2_counter_collection.csv > $D/summary.txt; cat $D/summary.txt | cut -c1-300 ;;
    pmc-c3) bash tools/gpu_pmc_config.sh r06 c3 || exit $? ;;
    pmc-inst) bash tools/gpu_pmc_config.sh r06 c3_two_level --instancing two-level || exit $? ;;
    pmc-c5) bash tools/gpu_pmc_config.sh r06 c5 --workload c5 --width 1920 --height 1080 --spp 1024 || exit $? ;;
    pmc-e8) bash tools/gpu_pmc_config.sh r06 c4_share8 --emulate-ranks 8 || exit $? ;;
    pmc-c2) bash tools/gpu_pmc_config.sh r06 c2 --workload cbox || exit $? ;;
    *) echo "unknown step $w"; exit 2 ;;
  esac
done
