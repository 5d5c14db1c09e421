#!/bin/bash
# round 6: f32 decoder weight-gradient deferral on the final tree
bash tools/gpurun/ab.sh r06zn 3 "" base "SEG_WGRAD_DEFER=52:51" "SEG_WGRAD_DEFER=52:30" || exit 1
