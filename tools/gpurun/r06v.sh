#!/bin/bash
# round 6: all-points Winograd weight gradient (seg_conv_wino_wgrad16): parity + per-launch timing, tile variants
d=gpurun_out/r06v; mkdir -p $d
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "wino_wgrad" -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1 || { tail -30 $d/tests.log; exit 1; }
tail -2 $d/tests.log
timeout -k 10 200 python -u tools/ww16bench.py > $d/mnv2.txt 2>&1 || { tail -20 $d/mnv2.txt; exit 1; }
cat $d/mnv2.txt
for v in ww32 ww64; do
  SEG_LIB_PATH=variants/$v.so timeout -k 10 200 python -u tools/ww16bench.py > $d/mnv2_$v.txt 2>&1 || { tail -20 $d/mnv2_$v.txt; exit 1; }
  echo "== $v"; cat $d/mnv2_$v.txt
done
timeout -k 10 300 python -u tools/ww16bench.py unet > $d/unet.txt 2>&1 || { tail -20 $d/unet.txt; exit 1; }
cat $d/unet.txt
