#!/bin/bash
# PMC passes over the ICP (C4) workload (one rocprofv3 run per pass; no
# --pmc is ever combined with sys/runtime tracing).  Usage: scripts/pmc_icp.sh TAG [CFG unused] [CELL]
# PMC_SCRIPT (default scripts/icp_cells.py CELL) and PMC_FILTER (kernel-name regex, default icp) select
# another workload, e.g. the fidelity statistics: PMC_SCRIPT="scripts/icp_ab.py 1.0 1" PMC_FILTER="seq_|pcl_"
set -u
TAG=${1:-pmc}; CFG=${2:-C2}; CELL=${3:-1.0}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
while read -r ctrs; do
    [ -z "$ctrs" ] && continue
    i=$((i + 1))
    echo "== pass $i: $ctrs"
    timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace -d "$OUT/p$i" -o run --output-format csv \
        -- python ${PMC_SCRIPT:-scripts/icp_cells.py $CELL} > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done <<'EOF'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_WR
SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_MISC
FETCH_SIZE
WRITE_SIZE
EOF
python - "$OUT" "${PMC_FILTER:-icp}" <<'PY'
import csv, glob, os, re, sys, collections
out, filt = sys.argv[1], re.compile(sys.argv[2])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:64]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if not filt.search(k):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:34s} mean/dispatch {sum(v)/len(v):14.1f}  n={len(v)}")
PY
