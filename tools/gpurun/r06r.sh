#!/bin/bash
# round 6: per-CU occupancy cap of the side stream's weight-gradient kernels (dynamic LDS pad) -- step A/B
t=${1:-r06r}
export TMPDIR=/tmp
bash tools/gpurun/ab.sh $t 2 "--math f32" base "SEG_SIDE_LDS_PAD=16384" "SEG_SIDE_LDS_PAD=32768" "SEG_SIDE_LDS_PAD=49152" "SEG_SIDE_LDS_PAD=65536" || exit 1
bash tools/gpurun/ab.sh $t 2 "--math bf16io" base "SEG_SIDE_LDS_PAD=16384" "SEG_SIDE_LDS_PAD=32768" "SEG_SIDE_LDS_PAD=49152" || exit 1
cat gpurun_out/$t/ab.txt
