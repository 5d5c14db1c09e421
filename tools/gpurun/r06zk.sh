#!/bin/bash
# round 6: bf16 weight-gradient block target 512 (as built) vs 256 / 1024 on the final tree
bash tools/gpurun/ab.sh r06zk 3 "--math bf16io" base "lib=variants/wbb256.so" "lib=variants/wbb1024.so" || exit 1
bash tools/gpurun/ab.sh r06zk 2 "--model UNet --height 512 --width 1024 --batch 8 --math bf16io" base "lib=variants/wbb256.so" || exit 1
