#!/bin/bash
# A/B two builds of libsegamd.so on one box: bash tools/ab_lib.sh <other.so> [bench args]
other=$1; shift
for i in 1 2; do
  for lib in "" "$other"; do
    SEG_LIB_PATH=${lib:-team02-objectdetection_amd/seg_amd/_lib/libsegamd.so} timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timer "$@" > gpurun_out/abl.log 2>&1 || { echo "failed"; tail -3 gpurun_out/abl.log; exit 1; }
    echo "lib=${lib:-new} $(grep -o '"value": [0-9.]*' gpurun_out/abl.log)"
  done
done
