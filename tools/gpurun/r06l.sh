#!/bin/bash
# round 6: igemm2 interleaved-DMA K loop -- bitwise tests, per-launch A/B on the UNet / MobileNetV2UNet shapes,
# step A/B (UNet configs[4] bf16io, MobileNetV2UNet bf16io); then the side-stream diagnostic (r06k)
t=${1:-r06l}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_igemm2.py > $d/pytest.log 2>&1
rc=$?; tail -2 $d/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $d/pytest.log | head -20; exit $rc; }
for il in 0 1; do
  SEG_IG2_IL=$il timeout -k 10 300 python tools/ig2bench.py --set unet --kernel ig2 --reps 10 > $d/ig2_unet_il$il.txt 2>&1 || { tail -5 $d/ig2_unet_il$il.txt; exit 1; }
  SEG_IG2_IL=$il timeout -k 10 300 python tools/ig2bench.py --set mnv2 --kernel ig2 --reps 20 > $d/ig2_mnv2_il$il.txt 2>&1 || { tail -5 $d/ig2_mnv2_il$il.txt; exit 1; }
done
paste $d/ig2_unet_il0.txt $d/ig2_unet_il1.txt | head -40
bash tools/gpurun/ab.sh $t 2 "--model UNet --height 512 --width 1024 --batch 8 --math bf16io" base "SEG_IG2_IL=0" || exit 1
bash tools/gpurun/ab.sh $t 2 "--math bf16io" base "SEG_IG2_IL=0" || exit 1
bash tools/gpurun/r06k.sh ${t}_k
