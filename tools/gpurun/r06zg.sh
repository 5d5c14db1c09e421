#!/bin/bash
# round 6: all-points Winograd weight gradient on the 32x32 tile everywhere (2 blocks/CU, 216 regs) vs 64x64 for >= 128 channels
bash tools/gpurun/ab.sh r06zg 3 "" base "lib=variants/ww32.so" || exit 1
bash tools/gpurun/ab.sh r06zg 2 "--model UNet --height 512 --width 1024 --batch 8" base "lib=variants/ww32.so" || exit 1
