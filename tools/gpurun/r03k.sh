#!/bin/bash
# Round-3 pass k: exact-zero conv-bias gradients before BatchNorm (suite + A/B), igemm2 at step level
# (MobileNetV2UNet) and per launch (UNet 512x1024).
t=r03k
U="--model UNet --height 512 --width 1024 --batch 8"
bash tools/gpurun/steps.sh $t \
  "pytest|400|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "ab_mnv2|500|bash tools/gpurun/ab.sh ${t}_mnv2 3 '--math bf16io' base SEG_IGEMM2=0 SEG_ZERO_BN_BIAS=0" \
  "ab_unet|400|bash tools/gpurun/ab.sh ${t}_unet 2 '--math bf16io $U' base SEG_ZERO_BN_BIAS=0" \
  "tp_unet|200|SEG_OVERLAP=0 python tools/tapeprof.py --math bf16io $U --steps 3 --top 60 --csv gpurun_out/$t/tp_unet.csv" \
  "tp_unet_noig2|200|SEG_OVERLAP=0 SEG_IGEMM2=0 python tools/tapeprof.py --math bf16io $U --steps 3 --top 60 --csv gpurun_out/$t/tp_unet_noig2.csv"
