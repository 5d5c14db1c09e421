#!/bin/bash
# round 6: wino_wgrad16 with branch-free buffer loads (per-block bases, offsets computed before the loads)
d=gpurun_out/r06ze; mkdir -p $d
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "wino_wgrad" -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1 || { tail -30 $d/tests.log; exit 1; }
tail -1 $d/tests.log
timeout -k 10 200 python -u tools/ww16bench.py > $d/mnv2.txt 2>&1 || { tail -20 $d/mnv2.txt; exit 1; }
cat $d/mnv2.txt
SEG_LIB_PATH=variants/ww16old.so timeout -k 10 200 python -u tools/ww16bench.py > $d/mnv2_old.txt 2>&1 || { tail -20 $d/mnv2_old.txt; exit 1; }
cat $d/mnv2_old.txt
bash tools/gpurun/ab.sh r06ze 3 "" base "lib=variants/ww16old.so" || exit 1
bash tools/gpurun/ab.sh r06ze 2 "--model UNet --height 512 --width 1024 --batch 8" base "lib=variants/ww16old.so" || exit 1
