#!/bin/bash
# round 6: f32 decoder weight-gradient deferral on the wino_wgrad16 tree (and with the 1024-block direct wgrad)
bash tools/gpurun/ab.sh r06zc 3 "" base "SEG_WGRAD_DEFER=52:51" "SEG_WGRAD_DEFER=52:51 lib=variants/wb1024.so" "lib=variants/wb1024.so" || exit 1
