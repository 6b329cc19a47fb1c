#!/bin/bash
# A/B of one environment switch on the GPU box: parity tests + kNN timing + bench per value.
# usage: scripts/ab_env.sh <tag> <VAR> <v1> [v2 ...]
set -u
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in "$@"; do
    export "$VAR=$v"
    echo "== $VAR=$v"
    timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
        > "$OUT/parity_$v.log" 2>&1; rc=$?
    tail -n 2 "$OUT/parity_$v.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!! rc=$rc"; exit $rc; fi
    timeout -k 10 300 python scripts/knn_timing.py C3 > "$OUT/knn_$v.log" 2>&1 || exit $?
    cat "$OUT/knn_$v.log"
    timeout -k 10 300 python bench.py --steps 400 --warmup 20 --no-icp --no-cpu --streams '' > "$OUT/bench_$v.log" 2>&1 || exit $?
    python3 -c "import json,sys;d=json.loads([l for l in open('$OUT/bench_$v.log') if l.startswith('{')][-1]);r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'near',r['near_kernel_avg_ms'],'far',r['far_kernel_avg_ms'],'plane',r['plane_kernel_avg_ms'],'reuse',r['reuse_kernel_avg_ms'])"
done
