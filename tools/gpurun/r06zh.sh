#!/bin/bash
# round 6: fp32 direct weight gradient with 32-pixel K steps (vs 16)
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06zh_tests.log 2>&1; tail -1 gpurun_out/r06zh_tests.log
SEG_LIB_PATH=variants/wbk32.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06zh_tests_v.log 2>&1 || { tail -20 gpurun_out/r06zh_tests_v.log; exit 1; }
tail -1 gpurun_out/r06zh_tests_v.log
bash tools/gpurun/ab.sh r06zh 3 "" base "lib=variants/wbk32.so" || exit 1
bash tools/gpurun/ab.sh r06zh 2 "--model UNet --height 512 --width 1024 --batch 8" base "lib=variants/wbk32.so" || exit 1
