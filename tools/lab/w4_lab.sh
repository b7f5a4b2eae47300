#!/bin/bash
# gemm_w4 lab.  Build on the CPU container:  tools/lab/w4_lab.sh build <name> [extra hipcc flags]
#               Run on the GPU box:          tools/lab/w4_lab.sh run <out.jsonl> <name>...
set -e
if [ "$1" != build ]; then out=$(realpath -m "$2"); fi
cd "$(dirname "$0")"
if [ "$1" = build ]; then
  name=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 "$@" w4_lab.hip -o w4_lab_$name 2>/dev/null
  ls -la w4_lab_$name
else
  shift 2
  mkdir -p "$(dirname "$out")"
  SHAPES=("512 8192 3584" "512 28672 3584" "2048 3584 4096" "2048 8192 3584" "2048 256000 3584" "4096 28672 3584" "4096 3584 14336" "8192 8192 3584")
  for name in "$@"; do
    echo "{\"build\": \"$name\"}" >> "$out"
    timeout -k 5 120 ./w4_lab_$name check >> "$out"
    for shp in "${SHAPES[@]}"; do
      timeout -k 5 60 ./w4_lab_$name time $shp 10 >> "$out"
    done
  done
fi
