#!/bin/bash
# Round-3 pass d: the one-launch small-layer BN backward (grid barriers): its kernel test
# first, the model suites with it on, per-launch profile, interleaved A/B.
t=r03d
bash tools/gpurun/steps.sh $t \
  "bn_small|120|python -u -m pytest tests/test_gpu_bn_small.py -x -q --timeout 60 --timeout-method thread" \
  "pytest_small|400|SEG_BN_SMALL=16777216 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_tape.py tests/test_gpu_configs.py tests/test_gpu_bf16io.py tests/test_gpu_ddp.py -x -q --timeout 300 --timeout-method thread" \
  "tp_bf16io_small|300|SEG_OVERLAP=0 SEG_BN_SMALL=16777216 python tools/tapeprof.py --math bf16io --top 100 --csv gpurun_out/$t/tp_bf16io_small.csv" \
  "ab_bf16io|500|bash tools/gpurun/ab.sh ${t}_bf16io 3 '--math bf16io' base SEG_BN_SMALL=16777216" \
  "ab_f32|500|bash tools/gpurun/ab.sh ${t}_f32 3 '--math f32' base SEG_BN_SMALL=16777216"
