#!/bin/bash
# Round-3 A/Bs (interleaved, one box): igemm2 on/off, 8-row BN reductions, BX dgrads.
t=r03b
bash tools/gpurun/steps.sh $t \
  "ab_bf16io|900|bash tools/gpurun/ab.sh ${t}_bf16io 2 '--math bf16io' base SEG_BX=1 SEG_IGEMM2=0 lib=variants/chan8.so" \
  "ab_f32|600|bash tools/gpurun/ab.sh ${t}_f32 2 '--math f32' base SEG_BX=1 lib=variants/chan8.so"
