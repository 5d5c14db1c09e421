#!/bin/bash
# upsample-fold diagnostics: the new kernel tests verbose, no -x
d=gpurun_out/r06c; mkdir -p $d
timeout -k 10 300 python -u -m pytest -q -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mbconv.py -k "upsample_fold" > $d/pytest.log 2>&1
grep -E "upsample fold|passed|failed|Error" $d/pytest.log | head -30
