#!/bin/bash
# side-cap + BIN correctness, then interleaved A/B of SEG_SIDE_CAP and SEG_BIN_DW
t=${1:-r05c}
d=gpurun_out/$t; mkdir -p $d
bash tools/gpurun/steps.sh $t \
  "captest|300|python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bin.py -k 'side_cap or bin' -x -q --timeout 120 --timeout-method thread" \
  "capmodel|300|SEG_SIDE_CAP=256 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_wgrad2.py tests/test_gpu_tape.py -x -q --timeout 120 --timeout-method thread" || exit 1
grep -q passed $d/captest.log && ! grep -q failed $d/captest.log && grep -q passed $d/capmodel.log && ! grep -q failed $d/capmodel.log || exit 1
bash tools/gpurun/ab.sh ${t}_bf16io 2 "--math bf16io" "SEG_BIN_DW=0" base "SEG_SIDE_CAP=256" "SEG_SIDE_CAP=512" || exit 1
bash tools/gpurun/ab.sh ${t}_f32 2 "--math f32" "SEG_BIN_DW=0" base "SEG_SIDE_CAP=256" "SEG_SIDE_CAP=512" || exit 1
