#!/bin/bash
# round 6: the 1024-block f32 direct weight gradient on UNet 512x1024 f32
bash tools/gpurun/ab.sh r06zd 2 "--model UNet --height 512 --width 1024 --batch 8" base "lib=variants/wb1024.so" || exit 1
