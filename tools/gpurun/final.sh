#!/bin/bash
# end-of-round evidence: rocprofv3 roofline profiles (kernel trace + FETCH/WRITE/MFMA PMC) of f32 and bf16io,
# the default bench line (with the CPU baseline), the bf16io line and configs[4] (UNet 512x1024 bs=8) lines
tag=$1
d=gpurun_out/$tag; mkdir -p $d
bash tools/gpurun/prof_pair.sh $tag || exit 1
timeout -k 10 300 python bench.py > $d/bench_f32.json 2> $d/bench_f32.err || { tail -5 $d/bench_f32.err; exit 1; }
timeout -k 10 300 python bench.py --math bf16io --steps 20 --warmup 5 --no-cpu-baseline > $d/bench_bf16io.json 2> $d/bench_bf16io.err || exit 1
bash tools/gpurun/unet_cfg5.sh ${tag}_unet || exit 1
tail -c 400 $d/bench_f32.json
