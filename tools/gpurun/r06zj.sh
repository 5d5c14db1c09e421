#!/bin/bash
# round 6: direct weight gradient with two register sets (loads two K steps ahead) vs one
d=gpurun_out/r06zj; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bf16io.py tests/test_gpu_bf16.py tests/test_gpu_wgrad2.py tests/test_gpu_model.py tests/test_gpu_tape.py -x -q --timeout 300 --timeout-method thread > $d/tests.log 2>&1 || { tail -30 $d/tests.log; exit 1; }
tail -1 $d/tests.log
bash tools/gpurun/ab.sh r06zj 3 "" base "lib=variants/pf1.so" || exit 1
bash tools/gpurun/ab.sh r06zj 3 "--math bf16io" base "lib=variants/pf1.so" || exit 1
bash tools/gpurun/ab.sh r06zj 2 "--model UNet --height 512 --width 1024 --batch 8 --math bf16io" base "lib=variants/pf1.so" || exit 1
