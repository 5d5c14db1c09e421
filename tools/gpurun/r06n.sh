#!/bin/bash
# round 6: which weight gradients cost the step -- skip subsets (diagnostic only): the encoder's high-resolution
# tail (ops 0-9), the rest of the encoder (10-51), the decoder (52-66)
t=${1:-r06n}
export TMPDIR=/tmp
bash tools/gpurun/ab.sh $t 2 "--math bf16io" base "SEG_DIAG_SKIP_WGRAD=0:10" "SEG_DIAG_SKIP_WGRAD=10:52" "SEG_DIAG_SKIP_WGRAD=52:70" || exit 1
bash tools/gpurun/ab.sh $t 1 "--math f32" base "SEG_DIAG_SKIP_WGRAD=0:10" "SEG_DIAG_SKIP_WGRAD=10:52" "SEG_DIAG_SKIP_WGRAD=52:70" || exit 1
cat gpurun_out/$t/ab.txt
