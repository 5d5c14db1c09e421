#!/bin/bash
# deferred weight-gradient fork: parity with it on, then interleaved A/B
t=${1:-r05d}
d=gpurun_out/$t; mkdir -p $d
bash tools/gpurun/steps.sh $t \
  "defer|300|SEG_WGRAD_DEFER=1 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_tape.py tests/test_gpu_ddp.py -x -q --timeout 120 --timeout-method thread" || exit 1
grep -q passed $d/defer.log && ! grep -q failed $d/defer.log || exit 1
bash tools/gpurun/ab.sh ${t}_bf16io 3 "--math bf16io" base "SEG_WGRAD_DEFER=1" || exit 1
bash tools/gpurun/ab.sh ${t}_f32 3 "--math f32" base "SEG_WGRAD_DEFER=1" || exit 1
