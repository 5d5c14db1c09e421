#!/bin/bash
# round 6, first box: regression check at HEAD, UNet configs[4] side stream on/off A/B,
# SQ counter passes over the bf16 dense 3x3 kernels (item 2)
t=${1:-r06a}
export TMPDIR=/tmp
mkdir -p gpurun_out/$t
timeout -k 10 60 rocprofv3 -L > gpurun_out/$t/counters.txt 2>&1
bash tools/gpurun/check.sh $t || exit 1
bash tools/gpurun/ab.sh ${t}_ab 2 "--model UNet --height 512 --width 1024 --batch 8 --math bf16io" base "SEG_OVERLAP=0" || exit 1
bash tools/gpurun/ab.sh ${t}_ab 2 "--model UNet --height 512 --width 1024 --batch 8 --math f32" base "SEG_OVERLAP=0" || exit 1
bash tools/gpurun/sq.sh ${t}_sq_unet --model UNet --height 512 --width 1024 --batch 8 --math bf16io || exit 1
bash tools/gpurun/sq.sh ${t}_sq_mnv2 --math bf16io || exit 1
