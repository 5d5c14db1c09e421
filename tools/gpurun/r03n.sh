#!/bin/bash
# Round-3 pass n: engine knobs tuned on MobileNetV2UNet, re-checked on UNet 512x1024 (configs[4]).
t=r03n
U="--model UNet --height 512 --width 1024 --batch 8"
bash tools/gpurun/steps.sh $t \
  "ab_unet_bf16io|700|bash tools/gpurun/ab.sh ${t}_ub 2 '--math bf16io $U' base SEG_HALO_BF16=0 SEG_IGEMM2_MAX_ROWS=262144 SEG_FORK_LATE=0" \
  "ab_unet_f32|500|bash tools/gpurun/ab.sh ${t}_uf 2 '--math f32 $U' base SEG_WINO_WGRAD=0"
