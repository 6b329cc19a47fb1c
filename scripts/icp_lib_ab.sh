#!/bin/bash
# ICP tile-order A/B (GPU box): default (64 interleaved segments) vs cost-balanced contiguous XCD shares
# in later passes (contig1) and in every pass (contig2).  Per variant: parity (ICP tests), 2 x 5 alignments
# per pair (scripts/icp_ab.py), FETCH_SIZE / WRITE_SIZE per icp_tile_kernel dispatch.
# usage: [NOPMC=1] scripts/icp_contig_ab.sh <outdir> [variants...]   (variant: default = the in-tree build, else build_ab/<name>)
set -u
OUT=${1:-gpurun_out/icpab}; shift || true
VARS=${*:-"default contig1 contig2"}
mkdir -p "$OUT"
export TMPDIR=/tmp
lib() { [ "$1" = default ] && echo "" || echo "fast-lio-sam_gps_amd/build_ab/$1/liblio_gpu.so"; }
step() {  # step <name> <seconds> <cmd...>: any non-zero exit ends the script
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
    [ $rc -eq 0 ] || exit $rc
}
for v in $VARS; do
    export LIO_GPU_LIB=$(lib $v)
    step "test_$v" 300 python -u -m pytest tests/test_gpu_icp.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
done
for r in 1 2; do
    for v in $VARS; do
        export LIO_GPU_LIB=$(lib $v)
        step "time_${v}_$r" 200 python scripts/icp_ab.py 1.0 5
    done
done
[ -n "${NOPMC:-}" ] && { echo "icp ab done (no PMC)"; exit 0; }
for v in $VARS; do
    export LIO_GPU_LIB=$(lib $v)
    for c in FETCH_SIZE WRITE_SIZE; do
        step "pmc_${v}_$c" 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_${v}_$c" -o run --output-format csv \
            -- python scripts/icp_ab.py 1.0 1
    done
done
python - "$OUT" $VARS <<'PY'
import csv, glob, os, sys, statistics
out, vars_ = sys.argv[1], sys.argv[2:]
for v in vars_:
    row = [v]
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = []
        for f in glob.glob(os.path.join(out, f"pmc_{v}_{c}", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "icp_tile_kernel" in r.get("Kernel_Name", "") and r["Counter_Name"] == c:
                    vals.append(float(r["Counter_Value"]))
        row.append(f"{c} mean {statistics.mean(vals) / 1024:.0f} KiB/dispatch over {len(vals)}" if vals else f"{c} none")
    print(" | ".join(row))
PY
echo "icp ab done"
