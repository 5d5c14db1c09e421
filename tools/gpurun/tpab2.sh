#!/bin/bash
# per-launch profiles (no side stream) of the default library and each variants/*.so on one workload:
# tpab2.sh <tag> <math> [tapeprof args]
tag=$1; math=$2; shift 2
d=gpurun_out/$tag; mkdir -p $d
for lib in team02-objectdetection_amd/seg_amd/_lib/libsegamd.so variants/*.so; do
  n=$(basename $lib .so)
  SEG_LIB_PATH=$lib SEG_OVERLAP=0 timeout -k 10 300 python tools/tapeprof.py --math $math --top 400 "$@" > $d/tp_$n.txt 2>&1 || { echo "$lib failed"; tail -5 $d/tp_$n.txt; exit 1; }
done
