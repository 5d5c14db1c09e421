#!/bin/bash
# End-of-round evidence, part 2: the default bench line (f32 headline + nested bf16io / infer / unet_cfg5
# blocks + CPU baseline) and configs[4]'s own lines.
set -o pipefail
tag=$1
d=gpurun_out/$tag; mkdir -p $d
export SEG_COMMIT=$(cat .commit 2>/dev/null)
timeout -k 10 500 python bench.py > $d/bench.json 2> $d/bench.err || { tail -5 $d/bench.err; exit 1; }
bash tools/gpurun/unet_cfg5.sh ${tag}_unet || exit 1
tail -c 600 $d/bench.json
