#!/bin/bash
# round 6: two-stream timeline of the final tree (f32, bf16io)
d=gpurun_out/r06zi; mkdir -p $d
timeout -k 10 240 python -u tools/timeline.py --math f32 --steps 6 > $d/tl_f32.txt 2>&1 || { tail -20 $d/tl_f32.txt; exit 1; }
timeout -k 10 240 python -u tools/timeline.py --math bf16io --steps 6 > $d/tl_bf16io.txt 2>&1 || { tail -20 $d/tl_bf16io.txt; exit 1; }
grep -A8 "^tape of 3" $d/tl_f32.txt; grep -A8 "^tape of 3" $d/tl_bf16io.txt
