#!/bin/bash
# A/B of HIP runtime knobs on the C2 bench (launch latency): each run under its own time limit,
# stop at the first failure.
set -u
OUT=gpurun_out/${1:-envab}
mkdir -p "$OUT"
run() {  # run <name> <env...> -- (bench args fixed)
    local name=$1; shift
    echo "== $name"
    timeout -k 10 300 env "$@" python bench.py --steps 400 --warmup 40 --no-icp --no-cpu > "$OUT/$name.log" 2>&1
    local rc=$?
    grep '^{' "$OUT/$name.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], d['capi_ms_per_scan'])"
    [ $rc -eq 0 ] || { echo "rc=$rc, stopping"; exit $rc; }
}
run base X=0 &&
run devkernarg HIP_FORCE_DEV_KERNARG=1 &&
run base2 X=0 &&
run devkernarg2 HIP_FORCE_DEV_KERNARG=1
