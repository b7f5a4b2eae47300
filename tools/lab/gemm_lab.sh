#!/bin/bash
# Build (on the CPU container) one gemm_lab executable per knob setting: tools/lab/gemm_lab.sh build
# Run them on the GPU box:                                                tools/lab/gemm_lab.sh run
set -e
cd "$(dirname "$0")"
VARIANTS=("base:" "m32:-DPP_MFMA32=1" "nolds:-DPP_NO_LDS_READ=1")
if [ "$1" = build ]; then
  for v in "${VARIANTS[@]}"; do
    name=${v%%:*}; flags=${v#*:}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 $flags gemm_lab.hip -o gemm_lab_$name &
  done
  wait
  ls -la gemm_lab_*
else
  mkdir -p ../../gpurun_out
  for v in "${VARIANTS[@]}"; do
    name=${v%%:*}
    for shp in "4096 28672 3584 0" "4096 28672 3584 3" "4096 8192 3584 0" "2048 28672 3584 3" "8192 8192 3584 0" "2048 256000 3584 0" "4096 3584 14336 0"; do
      echo -n "{\"variant\": \"$name\", \"r\": "; timeout -k 5 60 ./gemm_lab_$name $shp; echo "}"
    done
  done
fi
