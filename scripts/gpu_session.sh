#!/bin/bash
# GPU-box session: parity tests, smoke, bench, rocprof.  Each GPU step has its
# own time limit; any fault / abort / timeout (exit status other than 0 or 1)
# ends the session immediately — nothing else touches the GPU after it.
# usage: scripts/gpu_session.sh <tag> [steps...]   steps: test smoke bench prof pmc c3 c5 ppprof quick knn rehearse rccl
set -u
TAG=${1:-r01}; shift || true
STEPS=${*:-"test smoke bench prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo); cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null); affinity: $(python3 -c 'import os;print(len(os.sched_getaffinity(0)))')" | tee "$OUT/host.txt"

run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "!! $name ended with rc=$rc: stopping the session (no further GPU work)"
        exit $rc
    fi
    return 0
}

runs() {  # as run, but any failure (tests included) ends the session
    run "$@"
    grep -qE "(^| )(failed|error)" "$OUT/$1.log" && { echo "!! $1 had failures: stopping the session"; exit 1; }
    return 0
}

for s in $STEPS; do
    case $s in
    test)  run pytest_gpu 1100 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread ;;
    pipe)  runs pytest_pipe 600 python -u -m pytest tests/test_gpu_pipeline.py -x -v -s -p no:cacheprovider --timeout 500 --timeout-method thread ;;
    icpf)  runs pytest_icpf 600 python -u -m pytest tests/test_gpu_icp.py -k "float or double" -x -v -s -p no:cacheprovider --timeout 500 --timeout-method thread ;;
    icpx)  runs pytest_icpx 600 python -u -m pytest tests/test_gpu_icp.py -k "exchange or group" -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    spawn2) LIO_BENCH_REHEARSE=1 run spawn2 500 python bench.py --gpus 2 --steps 50 --warmup 5 --pipeline 0 --no-cpu --streams '' --icp-reps 2 ;;
    map)   runs pytest_map 900 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_fullsize.py -x -v -p no:cacheprovider --timeout 600 --timeout-method thread ;;
    shardt) runs pytest_shard 900 python -u -m pytest tests/test_gpu_icp.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py -k "group or exchange or emulated or multiprocess or recovery or timeout" -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread ;;
    shardprof) run shardprof4 300 env LIO_FSH_TRACE=1 python scripts/icp_shard_profile.py 4 3 B &&
               run shardprof8 300 python scripts/icp_shard_profile.py 8 2 B &&
               run shardtrace 300 rocprofv3 --kernel-trace --stats -d "$OUT/shardtrace" -o run --output-format csv -- python scripts/icp_shard_profile.py 4 2 B &&
               python scripts/icp_shard_kernels.py "$OUT/shardtrace/run_kernel_trace.csv" "$OUT/shard_kernels.txt" ;;
    shardrep) for wr in "4 1" "8 7"; do
                  set -- $wr
                  run shardrec$1 300 python scripts/icp_shard_replay.py record $1 $2 /tmp/rec$1.npz B &&
                  run shardrep$1 300 python scripts/icp_shard_replay.py replay $1 $2 /tmp/rec$1.npz 5 &&
                  run shardreptrace$1 300 rocprofv3 --kernel-trace --stats -d "$OUT/shardrep$1" -o run --output-format csv -- python scripts/icp_shard_replay.py replay $1 $2 /tmp/rec$1.npz 3 &&
                  python scripts/icp_shard_kernels.py "$OUT/shardrep$1/run_kernel_trace.csv" "$OUT/shardrep_kernels$1.txt"
              done ;;
    icpab) AB=${AB:-pre_fuse}
           run icpab 600 bash -c "for r in 1 2; do python scripts/icp_ab.py 1.0 5 && echo '^ new' && LIO_GPU_LIB=fast-lio-sam_gps_amd/build_ab/$AB/liblio_gpu.so python scripts/icp_ab.py 1.0 5 && echo '^ $AB' || exit \$?; done" &&
           run icpabtrace 300 rocprofv3 --kernel-trace --stats -d "$OUT/icpabtrace" -o run --output-format csv -- python scripts/icp_ab.py 1.0 1 &&
           python scripts/icp_tile_passes.py "$OUT/icpabtrace/run_kernel_trace.csv" new > "$OUT/tile_passes_new.txt" &&
           python scripts/kstats.py "$OUT/icpabtrace/run_kernel_stats.csv" > "$OUT/icpab_kstats.txt" ;;
    lseqab) run lseqgen 300 python -c "
import sys; sys.path.insert(0, 'fast-lio-sam_gps_amd')
from lio_gpu import pipeline as PL
kfs = PL.make_loop_keyframes(n_out=12, n_back=12); PL.write_loop_sequence('/tmp/ls.bin', kfs, range(12, 24))" &&
            for r in 1 2 3; do
                run lseq_new_$r 120 fast-lio-sam_gps_amd/lio_gpu/_lib/loop_sequence /tmp/ls.bin &&
                run lseq_pre_$r 120 fast-lio-sam_gps_amd/build_ab/lseq_pre/loop_sequence /tmp/ls.bin || exit $?
            done ;;
    lseqt) runs pytest_lseq 600 python -u -m pytest tests/test_cpp_stream.py tests/test_gpu_parity.py -k "loop_sequence or guard" -x -v -s -p no:cacheprovider --timeout 500 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    loopseqprof) run loopseqprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/loopseqprof" -o run --output-format csv -- fast-lio-sam_gps_amd/lio_gpu/_lib/loop_sequence /tmp/ls.bin &&
                 run loopseqapi 300 rocprofv3 --hip-runtime-trace --stats -d "$OUT/loopseqapi" -o run --output-format csv -- fast-lio-sam_gps_amd/lio_gpu/_lib/loop_sequence /tmp/ls.bin ;;
    loopseq) run loopseq 300 python -c "
import sys, json, tempfile, os; sys.path.insert(0, 'fast-lio-sam_gps_amd')
from lio_gpu import pipeline as PL
kfs = PL.make_loop_keyframes(n_out=12, n_back=12)
f = '/tmp/ls.bin'; PL.write_loop_sequence(f, kfs, range(12, 24))
o = PL.run_loop_sequence(f); pc = o.pop('per_call'); print(json.dumps(o))
for c in pc: print(c['k'], round(c['ms'], 3), round(c['submaps_ms'], 3), round(c['icp_ms'], 3), c['closest'], c['n_src'], c['n_dst'], c['iterations'], c['valid'], c['allocs'])
" ;;
    bench) run bench 600 python bench.py --steps 200 --warmup 20 ;;
    knn)   run knn_timing 300 python scripts/knn_timing.py C2 &&
           run knn_prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/knnprof" -o run --output-format csv -- python scripts/knn_timing.py C2 ;;
    quick) run bench_quick 400 python bench.py --steps 60 --warmup 5 --icp-reps 2 --cpu-scans 10 --cpu-warmup 2 ;;
    driver) run bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    driverq) run bench_driverq1 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --pipeline 0 --streams '' --no-icp &&
             run bench_driverq2 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --pipeline 0 --streams '' --no-icp &&
             run bench_driverq3 300 python bench.py --gpus 1 --steps 50 --warmup 5 --no-cpu --pipeline 0 --streams '' --no-icp ;;
    micro) run graph_cost 120 scripts/micro/graph_cost ;;
    first) run map_first 300 python scripts/map_first_call.py &&
           run map_first_nodefer 300 env HIP_ENABLE_DEFERRED_LOADING=0 python scripts/map_first_call.py ;;
    setup) run icp_setup 300 python scripts/icp_setup_timing.py &&
           run icp_setup2 300 python scripts/icp_setup_timing.py ;;
    msab)  echo "msab: the round-2 build it compared against is no longer kept (result: profiles/r04_multi_stream_ab.txt)" ;;
    pmcsq) run pmcsq_c3 300 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/pmcsq_c3" -o run --output-format csv -- python bench.py --steps 30 --warmup 3 --no-cpu --no-icp --streams '' --pipeline 0 &&
           run pmcsq_icp 300 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/pmcsq_icp" -o run --output-format csv -- python scripts/icp_ab.py 1.0 1 &&
           python scripts/pmc_sq_summary.py "$OUT/pmcsq_c3" "$OUT/pmcsq_c3.json" > "$OUT/pmcsq_c3_summary.txt" 2>&1;
           python scripts/pmc_sq_summary.py "$OUT/pmcsq_icp" "$OUT/pmcsq_icp.json" > "$OUT/pmcsq_icp_summary.txt" 2>&1; true ;;
    prep)  runs pytest_prep 600 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_formats.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread &&
           run prep_time 300 bash -c 'python scripts/prep_timing.py 80 && LIO_PREP_UPLOAD=full python scripts/prep_timing.py 80' &&
           run prep_profile 300 bash -c "LIO_PREP_PROFILE=1 python scripts/prep_timing.py 60 2> $OUT/prep_profile.err && python scripts/prep_profile_summary.py $OUT/prep_profile.err" &&
           run rocprof_prep 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof_prep" -o run --output-format csv -- python scripts/prep_timing.py 40 ;;
    sortab) runs pytest_prep_new 600 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_pipeline.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread &&
           run prep_ab 500 bash -c 'for r in 1 2 3; do python scripts/prep_timing.py 80 || exit $?; done' &&
           run prep_prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prep_prof" -o run --output-format csv -- python scripts/prep_timing.py 40 ;;
    setupfid) run icp_setup_fid 300 env LIO_ICP_ORDER=2 python scripts/icp_setup_timing.py &&
           run icp_setup_fid_b 300 env LIO_ICP_ORDER=2 python scripts/icp_setup_timing.py ;;
    c5prep) run c5_prep_profile 400 bash -c "LIO_PREP_PROFILE=1 python bench.py --config C5 --steps 20 --warmup 2 --no-icp --cpu-scans 2 --cpu-warmup 1 --pipeline 12 --streams '' > $OUT/c5prep.log 2> $OUT/c5prep.err && python scripts/prep_profile_summary.py $OUT/c5prep.err" ;;
    fidprof) run fid_prof 300 env LIO_ICP_ORDER=2 rocprofv3 --kernel-trace --stats -d "$OUT/fidprof" -o run --output-format csv -- python scripts/icp_ab.py 1.0 1 ;;
    maprec) runs pytest_maprec 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_pipeline.py -x -v -p no:cacheprovider --timeout 500 --timeout-method thread ;;
    fid)   runs pytest_fid 900 python -u -m pytest tests/test_gpu_seqsum.py tests/test_gpu_icp.py -k "seqsum or fidelity or double" -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread &&
           run icp_fid_time 300 env LIO_ICP_ORDER=2 python scripts/icp_ab.py 1.0 5 &&
           run icp_fid_time1 300 env LIO_ICP_ORDER=1 python scripts/icp_ab.py 1.0 3 ;;
    c3)    run bench_c3 600 python bench.py --config C3 --steps 60 --warmup 5 --no-icp --cpu-scans 10 --cpu-warmup 2 --pipeline 12 ;;
    c2)    run bench_c2 600 python bench.py --config C2 --steps 200 --warmup 20 --no-icp --cpu-scans 20 --cpu-warmup 2 --streams '' ;;
    c5)    run bench_c5 600 python bench.py --config C5 --steps 200 --warmup 20 --no-icp --cpu-scans 10 --cpu-warmup 2 --pipeline 12 --streams '' ;;
    ppprof) run rocprof_pipeline 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/ppprof" -o run \
               --output-format csv -- python bench.py --config C3 --steps 5 --warmup 2 --no-icp --no-cpu --pipeline 12 ;;
    rehearse) LIO_BENCH_REHEARSE=1 run rehearse2 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
               --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 --icp-reps 2 ;;
    prof)  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
               -- python bench.py --steps 100 --warmup 10 --no-cpu --icp-reps 3 --streams '' --pipeline 0 ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv \
               -- python bench.py --steps 30 --warmup 3 --no-cpu --no-icp --streams '' --pipeline 0 &&
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv \
               -- python bench.py --steps 30 --warmup 3 --no-cpu --no-icp --streams '' --pipeline 0 ;;
    pmcicp) run pmc_icp 900 bash scripts/pmc_icp.sh "$TAG/pmcicp" ;;
    pmcfid) PMC_SCRIPT="scripts/icp_ab.py 1.0 1" PMC_FILTER="seq_|pcl_" run pmc_fid 900 bash scripts/pmc_icp.sh "$TAG/pmcfid" ;;
    fullsize) run pytest_fullsize 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread ;;
    icptest) runs pytest_icp 600 python -u -m pytest tests/test_gpu_icp.py tests/test_gpu_parity.py -k icp -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    icppmc2) run icp_trace 300 rocprofv3 --kernel-trace -d "$OUT/icptrace" -o run --output-format csv -- python scripts/icp_ab.py 1.0 1 &&
             run icp_pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-trace -d "$OUT/icpsq" -o run --output-format csv -- python scripts/icp_ab.py 1.0 1 &&
             run icp_pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/icpfetch" -o run --output-format csv -- python scripts/icp_ab.py 1.0 1 &&
             run icp_pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/icpwrite" -o run --output-format csv -- python scripts/icp_ab.py 1.0 1 &&
             { python scripts/icp_pmc_traffic.py "$OUT" "$OUT/icp_traffic.json" > "$OUT/icp_traffic.txt" 2>&1; true; } ;;
    icpprof) run icp_prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/icpprof" -o run --output-format csv -- python scripts/icp_ab.py 1.0 1 &&
             run icp_pmc_valu 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace -d "$OUT/icppmc" -o run --output-format csv -- python scripts/icp_ab.py 1.0 1 ;;
    mapt)  run map_timing 400 python scripts/map_incr_timing.py 20 ;;
    mapprof) run map_prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/mapprof" -o run --output-format csv -- python scripts/map_incr_timing.py 20 ;;
    nearab) AB=${AB:-pre_near}
            run near_ab 600 bash -c "for r in 1 2 3; do python scripts/near_ab.py C3 && LIO_GPU_LIB=fast-lio-sam_gps_amd/build_ab/$AB/liblio_gpu.so python scripts/near_ab.py C3 || exit \$?; done" ;;
    parity) runs pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v -p no:cacheprovider --timeout 500 --timeout-method thread ;;
    icpseed) run icpseed_ab 600 bash -c 'for r in 1 2; do python scripts/icp_ab.py 1.0 5 && LIO_GPU_LIB=fast-lio-sam_gps_amd/build_ab/noseed/liblio_gpu.so python scripts/icp_ab.py 1.0 5 || exit $?; done' ;;
    icppre) run icppre_ab 900 bash -c 'for r in 1 2; do for v in default pre0 pre4 pre025; do if [ $v = default ]; then python scripts/icp_ab.py 1.0 5; else LIO_GPU_LIB=fast-lio-sam_gps_amd/build_ab/$v/liblio_gpu.so python scripts/icp_ab.py 1.0 5; fi || exit $?; echo "^ $v"; done; done' ;;
    icptrace) run icp_trace 300 rocprofv3 --kernel-trace -d "$OUT/icptrace" -o run --output-format csv -- python scripts/icp_ab.py 1.0 1 ;;
    rccl)  run rccl_one_gpu 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
               --master-port 29531 scripts/rccl_one_gpu.py ;;
    watchdog) LIO_BENCH_REHEARSE=1 run watchdog2 300 python bench.py --gpus 2 --steps 20 --warmup 2 --pipeline 0 --no-cpu --streams '' --icp-reps 1 --watchdog-s 0.5 ;;
    icp5)  runs pytest_icp5 900 python -u -m pytest tests/test_gpu_icp.py tests/test_gpu_dist.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "icp or ICP or sharded" -x -v -p no:cacheprovider --timeout 600 --timeout-method thread ;;
    icpt)  run icp_time2 300 python scripts/icp_ab.py 1.0 5 &&
           run icp_time_double 300 env LIO_ICP_ORDER=-1 python scripts/icp_ab.py 1.0 5 ;;
    knn5)  runs pytest_knn5 900 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_properties.py tests/test_gpu_map.py tests/test_gpu_fullsize.py tests/test_cpp_api.py -k "not icp" -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread ;;
    near5) run near5 600 bash -c 'for r in 1 2; do for c in C3 C2; do python scripts/near_ab.py $c && LIO_KNN_NEAR=cell python scripts/near_ab.py $c || exit $?; done; done' ;;
    cpps)  runs pytest_cpps 900 python -u -m pytest tests/test_cpp_stream.py tests/test_cpp_api.py -x -v -s -p no:cacheprovider --timeout 800 --timeout-method thread ;;
    mortab) run mortab 600 bash -c 'for r in 1 2; do for v in default cellorder; do if [ $v = default ]; then L=""; else L=fast-lio-sam_gps_amd/build_ab/$v/liblio_gpu.so; fi; LIO_GPU_LIB=$L LIO_ICP_ORDER=-1 python scripts/icp_ab.py 1.0 5 && LIO_GPU_LIB=$L python scripts/icp_ab.py 1.0 5 && LIO_GPU_LIB=$L LIO_ICP_ORDER=-1 python scripts/icp_ab.py 1.0 5 || exit $?; echo "^ $v round $r"; done; done' ;;
    libab) run libab 900 bash -c 'for r in 1 2; do for v in default $LIBAB; do if [ $v = default ]; then L=""; else L=fast-lio-sam_gps_amd/build_ab/$v/liblio_gpu.so; fi; LIO_GPU_LIB=$L python scripts/icp_ab.py 1.0 5 && LIO_GPU_LIB=$L LIO_ICP_ORDER=-1 python scripts/icp_ab.py 1.0 5 || exit $?; echo "^ $v round $r"; done; done' ;;
    abprof) run abprof_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/abprof_default" -o run --output-format csv -- python scripts/icp_ab.py 1.0 3 &&
            LIO_GPU_LIB=fast-lio-sam_gps_amd/build_ab/$LIBAB/liblio_gpu.so run abprof_ab 300 rocprofv3 --kernel-trace --stats -d "$OUT/abprof_ab" -o run --output-format csv -- python scripts/icp_ab.py 1.0 3 ;;
    abicp) run abicp 900 bash -c 'for r in 1 2; do for v in default $LIBAB; do if [ $v = default ]; then L=""; else L=fast-lio-sam_gps_amd/build_ab/$v/liblio_gpu.so; fi; LIO_GPU_LIB=$L LIO_ICP_ORDER=-1 python scripts/icp_ab.py 1.0 5 || exit $?; echo "^ $v round $r"; done; done' ;;
    cppprof) run cpp_prof 400 python scripts/cpp_stream_profile.py 3 ;;
    hwq)   run hwq 900 python scripts/hwq_ab.py ;;
    *) echo "unknown step $s" ;;
    esac
done
echo "session done"
