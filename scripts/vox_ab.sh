#!/bin/bash
# Build variants of liblio_gpu.so with vox_resolve_kernel experiment knobs (-DVOX_EXP=bits:
# 1 no counter atomics, 2 no tombstone pass, 4 no Add_Points sequence, 8 no map-side scan) into
# build_ab/voxN/ (CPU side), or time them on the GPU (run): map_incr_timing.py under rocprofv3.
set -eu
cd "$(dirname "$0")/../fast-lio-sam_gps_amd"
V=${VARIANTS:-"0 1 2 4 8 15"}
if [ "${1:-build}" = build ]; then
  for v in $V; do
    d=build_ab/vox$v; mkdir -p $d
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc -DVOX_EXP=$v -c csrc/lio_mapupd.hip -o $d/lio_mapupd.o
    objs=$(ls build/*.o | grep -v lio_mapupd.o)
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $d/liblio_gpu.so $objs $d/lio_mapupd.o -ldl -lpthread
  done
else
  cd ..
  export TMPDIR=/tmp
  for v in $V; do
    LIO_GPU_LIB=fast-lio-sam_gps_amd/build_ab/vox$v/liblio_gpu.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/voxab/v$v -o run --output-format csv -- python3 scripts/map_incr_timing.py 20 > gpurun_out/voxab_v$v.txt 2>&1
    python3 - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/voxab/v{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
d = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in csv.DictReader(open(f)) if "vox_resolve" in x["Kernel_Name"]]
d = sorted(d[1:])
print("variant", sys.argv[1], "vox_resolve us: median", d[len(d) // 2] / 1e3, "min", d[0] / 1e3, "max", d[-1] / 1e3)
PY
  done
fi
