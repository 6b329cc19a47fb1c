export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-icp --no-cpu --streams '' > gpurun_out/trace.log 2>&1 || exit $?
f=$(find gpurun_out/trace -name '*kernel_trace.csv' | head -1); cp $f gpurun_out/trace_kernels.csv; ls -la gpurun_out/trace_kernels.csv
