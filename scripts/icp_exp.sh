#!/bin/bash
# ICP (C4) tile-kernel sweep: target cell x tile cell, with ICP parity tests first.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/icpexp2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "icp or ICP or loop" -p no:cacheprovider > $OUT/parity.log 2>&1
rc=$?; tail -5 $OUT/parity.log; [ $rc -ne 0 ] && exit $rc
for tc in 2.0 3.0 1.5; do
  LIO_ICP_TILE_CELL=$tc timeout -k 10 200 python scripts/icp_cells.py 0.5,0.75,1.0,1.5,2.0 > $OUT/t$tc.log 2>&1 || exit $?
  echo "tile=$tc"; cat $OUT/t$tc.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python scripts/icp_cells.py 1.0 > $OUT/prof.log 2>&1 || exit $?
grep -h icp_ $(find $OUT/prof -name '*kernel_stats.csv') | cut -d, -f1-4
