#!/bin/bash
# side stream on (default) vs off, unprofiled, interleaved (the profiled bf16io step span was shorter with it off)
t=${1:-r05x}
bash tools/gpurun/ab.sh ${t} 2 "--math bf16io" base "SEG_OVERLAP=0" || exit 1
bash tools/gpurun/ab.sh ${t} 2 "--math f32" base "SEG_OVERLAP=0" || exit 1
cat gpurun_out/${t}/ab.txt
