#!/bin/bash
# configs[4] (UNet 10-class 512x1024 bs=8): bench lines (f32, bf16io) + a rocprofv3 kernel-stats profile of bf16io
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/$1; mkdir -p $d
for m in bf16io f32; do
  timeout -k 10 300 python bench.py --model UNet --height 512 --width 1024 --batch 8 --math $m --steps 10 --warmup 3 --no-cpu-baseline > $d/unet_$m.json 2> $d/unet_$m.err || { echo "bench $m failed"; tail -5 $d/unet_$m.err; exit 1; }
  tail -c 300 $d/unet_$m.json; echo
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d/prof -o run --output-format csv -- python bench.py --model UNet --height 512 --width 1024 --batch 8 --math bf16io --steps 5 --warmup 2 --no-cpu-baseline --no-timer > $d/prof.log 2>&1 || { echo "prof failed"; tail -5 $d/prof.log; exit 1; }
ls $d/prof
