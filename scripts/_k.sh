export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
for h in 0 120 160 220; do echo heavy=$h; LIO_KNN_HEAVY=$h timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kp$h -o run --output-format csv -- python scripts/knn_timing.py C2 2>&1 | grep 'shell hist'; grep -h -E 'near_kernel<false|far_kernel' $(find gpurun_out/kp$h -name '*kernel_stats.csv') | cut -d, -f1,4; done
