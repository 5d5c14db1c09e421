#!/bin/bash
# round 6: all-points Winograd weight gradient in the product: kernel tests, model suites, per-launch, f32 A/B
d=gpurun_out/r06x; mkdir -p $d
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "wino" -x -q --timeout 120 --timeout-method thread > $d/ops.log 2>&1 || { tail -30 $d/ops.log; exit 1; }
tail -1 $d/ops.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_unet_cfg5.py tests/test_gpu_tape.py tests/test_gpu_ddp.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $d/model.log 2>&1 || { tail -30 $d/model.log; exit 1; }
tail -1 $d/model.log
timeout -k 10 200 python -u tools/ww16bench.py > $d/mnv2.txt 2>&1 || { tail -20 $d/mnv2.txt; exit 1; }
cat $d/mnv2.txt
bash tools/gpurun/ab.sh r06x 3 "" base "SEG_WINO_WGRAD16=0" || exit 1
bash tools/gpurun/ab.sh r06x 2 "--model UNet --height 512 --width 1024 --batch 8" base "SEG_WINO_WGRAD16=0" || exit 1
