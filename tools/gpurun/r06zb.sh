#!/bin/bash
# round 6: f32 direct weight-gradient block target (2048 as built) against 512 / 1024 -- fewer rounds of side-stream blocks
bash tools/gpurun/ab.sh r06zb 3 "" base "lib=variants/wb512.so" "lib=variants/wb1024.so" || exit 1
