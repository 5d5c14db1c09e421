#!/bin/bash
# fused Winograd routed (seg_conv_wino_pick = 2): parity (ops, model, UNet cfg5, tape), per-shape timing on the
# MobileNetV2UNet and UNet 512x1024 decoder shapes, step A/B against the build without it; BN reduction shapes
# (fp32 4-channel lanes, 256-thread blocks) A/B
t=${1:-r05j}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
bash tools/gpurun/steps.sh $t \
  "tests|600|python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_unet_cfg5.py tests/test_gpu_tape.py -x -q --timeout 300 --timeout-method thread" || exit 1
grep -q passed $d/tests.log && ! grep -q failed $d/tests.log || exit 1
timeout -k 10 300 python -u tools/winobench.py > $d/winobench.txt 2>&1 || { tail -5 $d/winobench.txt; exit 1; }
WINOBENCH=unet timeout -k 10 400 python -u tools/winobench.py > $d/winobench_unet.txt 2>&1 || { tail -5 $d/winobench_unet.txt; exit 1; }
bash tools/gpurun/ab.sh ${t}_ab 2 "--math f32" base "lib=variants/nofused.so" "lib=variants/chanvw4.so" "lib=variants/red256.so" || exit 1
bash tools/gpurun/ab.sh ${t}_ab 2 "--math bf16io" base "lib=variants/red256.so" || exit 1
cat $d/winobench_unet.txt
