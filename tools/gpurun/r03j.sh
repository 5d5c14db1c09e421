#!/bin/bash
# Round-3 pass j: igemm2 scope -- MobileNetV2UNet bf16io with 1x1 convs on it too, and the
# UNet 512x1024 bf16io config with / without it.
t=r03j
bash tools/gpurun/steps.sh $t \
  "ab_mnv2|400|bash tools/gpurun/ab.sh ${t}_mnv2 2 '--math bf16io' base SEG_IGEMM2=all" \
  "ab_unet|600|bash tools/gpurun/ab.sh ${t}_unet 2 '--math bf16io --model UNet --height 512 --width 1024 --batch 8' base SEG_IGEMM2=0"
