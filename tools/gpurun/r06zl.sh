#!/bin/bash
# round 6: split sweep of the buffer-load all-points weight gradient (UNet 512x1024 and MobileNetV2UNet shapes)
d=gpurun_out/r06zl; mkdir -p $d
timeout -k 10 300 python -u tools/ww16sweep.py unet > $d/sweep_unet.txt 2>&1 || { tail -20 $d/sweep_unet.txt; exit 1; }
timeout -k 10 200 python -u tools/ww16sweep.py > $d/sweep_mnv2.txt 2>&1 || { tail -20 $d/sweep_mnv2.txt; exit 1; }
cat $d/sweep_unet.txt $d/sweep_mnv2.txt
