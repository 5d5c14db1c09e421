#!/bin/bash
# round 6: seg_conv_wino_wgrad16 split sweep (kernel / reduce apart), both tiles
d=gpurun_out/r06w; mkdir -p $d
timeout -k 10 200 python -u tools/ww16sweep.py > $d/sweep_mnv2.txt 2>&1 || { tail -20 $d/sweep_mnv2.txt; exit 1; }
SEG_LIB_PATH=variants/ww32.so timeout -k 10 200 python -u tools/ww16sweep.py > $d/sweep_mnv2_ww32.txt 2>&1 || { tail -20 $d/sweep_mnv2_ww32.txt; exit 1; }
timeout -k 10 300 python -u tools/ww16sweep.py unet > $d/sweep_unet.txt 2>&1 || { tail -20 $d/sweep_unet.txt; exit 1; }
SEG_LIB_PATH=variants/ww32.so timeout -k 10 300 python -u tools/ww16sweep.py unet > $d/sweep_unet_ww32.txt 2>&1 || { tail -20 $d/sweep_unet_ww32.txt; exit 1; }
cat $d/sweep_*.txt
