#!/bin/bash
# ICP (C4) tile-kernel check: exactness tests, then timing vs target cell size (tile cell via LIO_ICP_TILE_CELL).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/icpexp; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_icp.py tests/test_gpu_parity.py -q -m gpu -k "icp or ICP" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for tc in ${TILES:-2.0}; do echo tile=$tc; LIO_ICP_TILE_CELL=$tc timeout -k 10 120 python scripts/icp_cells.py ${CELLS:-0.75,1.0} 2>&1 | grep -E 'cell='; done
LIO_ICP_DEBUG=1 timeout -k 10 120 python scripts/icp_cells.py 1.0 2>&1 | grep -E 'dbg' | sort | uniq -c | head -3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python scripts/icp_cells.py 1.0 > $OUT/prof.log 2>&1 || exit $?
grep -h -E 'icp_|tile_' $(find $OUT/prof -name '*kernel_stats.csv') | cut -d, -f1-4
