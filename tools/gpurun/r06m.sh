#!/bin/bash
# round 6: the LDS-DMA bf16 weight gradient (csrc/wgrad3.hip) -- tests, per-launch against wgrad / wgrad2
t=${1:-r06m}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wgrad3.py > $d/pytest.log 2>&1
rc=$?; tail -2 $d/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $d/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python tools/wg3bench.py --set unet --reps 10 > $d/wg3_unet.txt 2>&1 || { tail -5 $d/wg3_unet.txt; exit 1; }
timeout -k 10 300 python tools/wg3bench.py --set mnv2 --reps 10 > $d/wg3_mnv2.txt 2>&1 || { tail -5 $d/wg3_mnv2.txt; exit 1; }
cat $d/wg3_unet.txt $d/wg3_mnv2.txt
