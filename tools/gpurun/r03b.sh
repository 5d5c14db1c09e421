#!/bin/bash
# Round-3 A/Bs (interleaved, one box): BX dgrads, 8-row BN reductions, igemm2 on/off,
# in-launch split-K combine of the inference convs.
t=r03b
bash tools/gpurun/steps.sh $t \
  "ab_infer|300|bash tools/gpurun/ab.sh ${t}_infer 3 '--workload infer --frames 300' base SEG_SPLITK_TK=0" \
  "ab_bf16io|800|bash tools/gpurun/ab.sh ${t}_bf16io 2 '--math bf16io' base SEG_BX=1 SEG_IGEMM2=0 lib=variants/chan8.so" \
  "ab_f32|600|bash tools/gpurun/ab.sh ${t}_f32 2 '--math f32' base SEG_BX=1 lib=variants/chan8.so"
