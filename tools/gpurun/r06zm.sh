#!/bin/bash
# round 6: side stream on / off on the final tree (unprofiled, interleaved)
bash tools/gpurun/ab.sh r06zm 3 "" base "SEG_OVERLAP=0" || exit 1
bash tools/gpurun/ab.sh r06zm 2 "--math bf16io" base "SEG_OVERLAP=0" || exit 1
bash tools/gpurun/ab.sh r06zm 2 "--model UNet --height 512 --width 1024 --batch 8" base "SEG_OVERLAP=0" || exit 1
