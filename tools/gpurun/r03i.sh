#!/bin/bash
# Round-3 pass i: the stem weight gradient's split count (the step's tail): interleaved A/B.
t=r03i
bash tools/gpurun/steps.sh $t \
  "ab_bf16io|500|bash tools/gpurun/ab.sh ${t}_bf16io 3 '--math bf16io' base SEG_STEM_SPLITS=4096 SEG_STEM_SPLITS=2048" \
  "ab_f32|500|bash tools/gpurun/ab.sh ${t}_f32 2 '--math f32' base SEG_STEM_SPLITS=4096 SEG_STEM_SPLITS=2048"
