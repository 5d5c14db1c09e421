#!/bin/bash
# round 6: the side stream's cost -- step time with the weight gradients skipped (diagnostic) and with overlap off
t=${1:-r06k}
export TMPDIR=/tmp
bash tools/gpurun/ab.sh $t 2 "--math bf16io" base "SEG_OVERLAP=0" "SEG_DIAG_SKIP_WGRAD=1" || exit 1
bash tools/gpurun/ab.sh $t 1 "--math f32" base "SEG_OVERLAP=0" "SEG_DIAG_SKIP_WGRAD=1" || exit 1
bash tools/gpurun/ab.sh $t 1 "--model UNet --height 512 --width 1024 --batch 8 --math bf16io" base "SEG_OVERLAP=0" "SEG_DIAG_SKIP_WGRAD=1" || exit 1
cat gpurun_out/$t/ab.txt
