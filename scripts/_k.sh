export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof -o run --output-format csv -- python scripts/knn_timing.py C2 > /dev/null 2>&1 || exit $?
grep -h -E 'plane|reuse|near|far' $(find gpurun_out/kprof -name '*kernel_stats.csv') | cut -d, -f1-4
for r in 1 2; do timeout -k 10 300 python bench.py --steps 1500 --warmup 50 --no-icp --no-cpu --streams '' 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['near_kernel_avg_ms'])"; done
