#!/bin/bash
# round 6: fp32 backward BN partials in one-row load groups (76 VGPRs, fits beside wino_wgrad16) vs four-row (148)
d=gpurun_out/r06z; mkdir -p $d
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16io.py tests/test_gpu_ops.py -k "chan or bn or partial or twin" -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1 || { tail -30 $d/tests.log; exit 1; }
tail -1 $d/tests.log
bash tools/gpurun/ab.sh r06z 3 "" base "lib=variants/rq4.so" || exit 1
bash tools/gpurun/ab.sh r06z 2 "--model UNet --height 512 --width 1024 --batch 8" base "lib=variants/rq4.so" || exit 1
