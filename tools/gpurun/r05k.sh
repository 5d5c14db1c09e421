#!/bin/bash
# full GPU suite + smoke at the fused-Winograd / BN-knob defaults, then step A/B against the pre-change build (r05old:
# 512-thread / 8-lane fp32 reductions, no fused Winograd), MobileNetV2UNet f32 + bf16io and UNet 512x1024 f32
t=${1:-r05k}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $d/pytest.log 2>&1 || { tail -15 $d/pytest.log; exit 1; }
tail -3 $d/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $d/smoke.log 2>&1 || { tail -5 $d/smoke.log; exit 1; }
tail -2 $d/smoke.log
bash tools/gpurun/ab.sh ${t}_ab 2 "--math f32" base "lib=variants/r05old.so" || exit 1
bash tools/gpurun/ab.sh ${t}_ab 2 "--math bf16io" base "lib=variants/r05old.so" || exit 1
bash tools/gpurun/ab.sh ${t}_ab 1 "--math f32 --model UNet --height 512 --width 1024 --batch 8 --steps 6 --warmup 2" base "lib=variants/r05old.so" || exit 1
cat ${d}_ab/ab.txt
