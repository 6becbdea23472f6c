#!/bin/bash
# Round-5 GPU call (one gpurun): the steps named on the command line, each under
# its own time limit; a failing step ends the call (test failures, pytest rc 1,
# excepted: the GPU is fine then and later steps still run).
#   tools/gpu_r05.sh [tests] [tests-new] [bench] [inst] [e8] [ranks] [c5] [c2] [kd] [pmc-*] [stats-*]
O=gpurun_out/r5
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 3 "$O/$name.log" | cut -c1-1500; if [ $rc -ne 0 ] && ! { [ "${name%%-*}" = tests ] && [ $rc -eq 1 ]; }; then exit $rc; fi; }
PYT="python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread"
for w in ${*:-tests bench}; do
  # a step may be repeated as name@k (its own log); the variant name drops the @k
  case $w in
    tests) step tests 900 $PYT tests ;;
    mathprobe) step mathprobe 300 tools/math_probe 3 ;;
    mathbench) step mathbench 120 tools/math_bench ;;
    mathprobe1) step mathprobe1 900 tools/math_probe 1 ;;
    tests-inst) step tests-inst 600 $PYT tests/test_gpu_instancing.py tests/test_gpu_edge_rays.py tests/test_gpu_finish.py ;;
    tests-entry) step tests-entry 600 $PYT tests/test_gpu_render_entry.py tests/test_gpu_edge_rays.py ;;
    tests-parity) step tests-parity 600 $PYT tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_c4.py ;;
    tests-kd) step tests-kd 600 $PYT tests/test_gpu_kdbuild.py ;;
    tests-new) step tests-new 600 $PYT tests/test_gpu_00_bench_ranks.py tests/test_gpu_c4.py tests/test_gpu_edge_rays.py ;;
    tests-builder) step tests-builder 600 $PYT tests/test_gpu_builder.py ;;
    tests-edge) step tests-edge 600 $PYT tests/test_gpu_edge_rays.py tests/test_gpu_kdbuild.py tests/test_gpu_instancing.py ;;
    tests-sfmt) step tests-sfmt 600 $PYT -s tests/test_gpu_rng_sfmt.py ;;
    tests-pp) step tests-pp 900 $PYT -s tests/test_gpu_parity.py tests/test_gpu_configs.py -k "roughconductor or rough_conductor or roughplastic or c5 or c1 or c2" ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 3 ;;
    quick*) step $w 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-parity --no-count ;;
    c5fin-*) v=${w#c5fin-}; step $w 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 --no-cpu --no-parity --no-count --finish-paths $v ;;
    c3fin-*) v=${w#c3fin-}; step $w 600 python bench.py --steps 10 --warmup 3 --no-cpu --no-parity --no-count --finish-paths $v ;;
    inst-quick*) step $w 300 python bench.py --steps 5 --warmup 2 --instancing two-level --no-cpu --no-parity --no-count ;;
    instvar-*) v=${w#instvar-}; v=${v%@*}; MTSG_LIB=my-mitsuba_amd/var/libmtsg_$v.so step $w 300 python bench.py --steps 5 --warmup 2 --instancing two-level --no-cpu --no-parity --no-count ;;
    c5bp-*) v=${w#c5bp-}; v=${v%@*}; step $w 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 --no-cpu --no-parity --no-count --batch-paths $v ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    refit-time) step refit-time 300 python -u -m pytest -m gpu -s -q tests/test_gpu_kdbuild.py -k "refit or c3_device" ;;
    c5quick*) step $w 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 --no-cpu --no-parity --no-count ;;
    c2quick) step c2quick 300 python bench.py --steps 5 --warmup 2 --workload cbox --no-cpu --no-parity --no-count ;;
    inst) step inst 300 python bench.py --steps 5 --warmup 2 --instancing two-level --no-cpu --no-parity ;;
    e8var-*) v=${w#e8var-}; v=${v%@*}; MTSG_LIB=my-mitsuba_amd/var/libmtsg_$v.so step $w 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 --no-cpu --no-parity --no-count ;;
    e8fin-*) v=${w#e8fin-}; v=${v%@*}; step $w 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 --no-cpu --no-parity --no-count --finish-paths $v ;;
    e8quick*) step $w 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 --no-cpu --no-parity --no-count ;;
    e8nb*) step $w 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 --no-cpu --no-parity --no-count --balance-rounds 0 ;;
    e8br-*) v=${w#e8br-}; v=${v%@*}; step $w 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 --no-cpu --no-parity --no-count --balance-rounds $v ;;
    tests-c4) step tests-c4 600 $PYT tests/test_gpu_c4.py tests/test_gpu_00_bench_ranks.py ;;
    e8) step e8 300 python bench.py --steps 5 --warmup 2 --emulate-ranks 8 --no-cpu --no-parity ;;
    ranks)
      # the launcher path (as the driver runs it) and the self-launching path,
      # two ranks on this one GPU; then the refusal without --allow-shared
      step ranks-torchrun 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --allow-shared
      step ranks-self 600 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --allow-shared
      echo "== ranks-refuse"; timeout -k 10 300 python bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu > $O/ranks-refuse.log 2>&1; echo "ranks-refuse rc=$? (non-zero expected)"; tail -n 2 $O/ranks-refuse.log ;;
    bench-ocml) MTSG_LIB=my-mitsuba_amd/var/libmtsg_ocmlmath.so step bench-ocml 600 python bench.py --steps 10 --warmup 3 --no-cpu ;;
    c5-ocml) MTSG_LIB=my-mitsuba_amd/var/libmtsg_ocmlmath.so step c5-ocml 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 --no-cpu ;;
    vtests-*) v=${w#vtests-}; MTSG_LIB=my-mitsuba_amd/var/libmtsg_$v.so step $w 600 $PYT tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edge_rays.py ;;
    var-*) v=${w#var-}; v=${v%@*}; MTSG_LIB=my-mitsuba_amd/var/libmtsg_$v.so step $w 600 python bench.py --steps 10 --warmup 3 --no-cpu --no-parity --no-count ;;
    c5var-*) v=${w#c5var-}; v=${v%@*}; MTSG_LIB=my-mitsuba_amd/var/libmtsg_$v.so step $w 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 --no-cpu --no-parity --no-count ;;
    c5) step c5 600 python bench.py --steps 3 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 ;;
    c2) step c2 600 python bench.py --steps 5 --warmup 2 --workload cbox ;;
    kd) step kd 300 python bench.py --steps 5 --warmup 2 --kd-build device --no-cpu --no-parity ;;
    stats-c3) step stats-c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-parity --no-count ;;
    stats-inst) step stats-inst 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_inst -o inst -- python3 bench.py --steps 5 --warmup 2 --instancing two-level --no-cpu --no-parity --no-count ;;
    stats-c5) step stats-c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 bench.py --steps 2 --warmup 1 --workload c5 --width 1920 --height 1080 --spp 1024 --no-cpu --no-parity --no-count ;;
    pmc-c3) bash tools/gpu_pmc_config.sh r05 c3 || exit $? ;;
    pmc-inst) bash tools/gpu_pmc_config.sh r05 c3_two_level --instancing two-level || exit $? ;;
    pmc-c5) bash tools/gpu_pmc_config.sh r05 c5 --workload c5 --width 1920 --height 1080 --spp 1024 || exit $? ;;
    pmc-e8) bash tools/gpu_pmc_config.sh r05 c4_share8 --emulate-ranks 8 || exit $? ;;
  esac
done
