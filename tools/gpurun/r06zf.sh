#!/bin/bash
# round 6: bf16 weight gradient with 64-pixel K steps (4 MFMA k-steps per load batch) vs 32
bash tools/gpurun/ab.sh r06zf 3 "--math bf16io" base "lib=variants/bkbf64.so" || exit 1
bash tools/gpurun/ab.sh r06zf 2 "--model UNet --height 512 --width 1024 --batch 8 --math bf16io" base "lib=variants/bkbf64.so" || exit 1
