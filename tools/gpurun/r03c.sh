#!/bin/bash
# Round-3 pass c: -m gpu suite, the model suites with SEG_BX=1, then interleaved A/Bs
# (in-launch split-K of the inference convs; BX dgrads and 8-row BN reductions, bf16io / f32).
t=r03c
bash tools/gpurun/steps.sh $t \
  "pytest|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "pytest_bx|400|SEG_BX=1 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_tape.py tests/test_gpu_configs.py tests/test_gpu_bf16io.py -x -q --timeout 300 --timeout-method thread" \
  "ab_infer|300|bash tools/gpurun/ab.sh ${t}_infer 3 '--workload infer --frames 300' base SEG_SPLITK_TK=0" \
  "ab_bf16io|500|bash tools/gpurun/ab.sh ${t}_bf16io 2 '--math bf16io' base SEG_BX=1 lib=variants/chan8.so" \
  "ab_f32|500|bash tools/gpurun/ab.sh ${t}_f32 2 '--math f32' base SEG_BX=1 lib=variants/chan8.so"
