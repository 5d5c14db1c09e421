#!/bin/bash
# rocprofv3 kernel stats of the current library and tmp_ab/libsegamd_old.so, f32 and bf16io
export TMPDIR=/tmp
mkdir -p gpurun_out
for math in f32 bf16io; do
  for lib in new old; do
    p=team02-objectdetection_amd/seg_amd/_lib/libsegamd.so; [ $lib = old ] && p=tmp_ab/libsegamd_old.so
    d=gpurun_out/abp_${lib}_${math}; mkdir -p $d
    SEG_LIB_PATH=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-timer --math $math > $d/bench.log 2>&1 || { echo "fail $lib $math"; tail -5 $d/bench.log; exit 1; }
    echo "$lib $math $(grep -o '"value": [0-9.]*' $d/bench.log)"
  done
done
