#!/bin/bash
# round 6: unprofiled two-stream timeline of the backward tape (tools/timeline.py), bf16io / f32 / UNet bf16io
d=gpurun_out/r06u; mkdir -p $d
timeout -k 10 240 python -u tools/timeline.py --math bf16io --steps 6 > $d/tl_bf16io.txt 2>&1 || { tail -20 $d/tl_bf16io.txt; exit 1; }
timeout -k 10 240 python -u tools/timeline.py --math f32 --steps 6 > $d/tl_f32.txt 2>&1 || { tail -20 $d/tl_f32.txt; exit 1; }
timeout -k 10 240 python -u tools/timeline.py --math bf16io --model UNet --height 512 --width 1024 --batch 8 --steps 4 > $d/tl_unet_bf16io.txt 2>&1 || { tail -20 $d/tl_unet_bf16io.txt; exit 1; }
cat $d/tl_bf16io.txt $d/tl_f32.txt $d/tl_unet_bf16io.txt
