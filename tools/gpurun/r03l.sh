#!/bin/bash
# Round-3 pass l: one-time zeroing of the conv biases' gradients before BN, igemm2 capped at 65k rows.
t=r03l
U="--model UNet --height 512 --width 1024 --batch 8"
bash tools/gpurun/steps.sh $t \
  "pytest|400|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "ab_mnv2|500|bash tools/gpurun/ab.sh ${t}_mnv2 3 '--math bf16io' base SEG_ZERO_BN_BIAS=0" \
  "ab_f32|400|bash tools/gpurun/ab.sh ${t}_f32 2 '--math f32' base SEG_ZERO_BN_BIAS=0" \
  "ab_unet|500|bash tools/gpurun/ab.sh ${t}_unet 2 '--math bf16io $U' base SEG_IGEMM2_MAX_ROWS=100000000 SEG_ZERO_BN_BIAS=0"
