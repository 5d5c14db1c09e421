#!/bin/bash
# short-lived weight-gradient blocks (4x the split count) against side-stream contention, interleaved
t=${1:-r05t}
bash tools/gpurun/ab.sh ${t} 2 "--math f32" base "lib=variants/wgblk8k.so" || exit 1
bash tools/gpurun/ab.sh ${t} 2 "--math bf16io" base "lib=variants/wgpx2k.so" || exit 1
cat gpurun_out/${t}/ab.txt
