#!/bin/bash
# End-of-round evidence: roofline profiles (kernel trace + FETCH/WRITE/MFMA PMC passes +
# per-queue breakdown) of f32 and bf16io, the default bench line (f32 headline + nested
# bf16io block + CPU baseline), and configs[4] (UNet 512x1024 bs=8) lines.
#   final.sh <tag>
set -o pipefail
tag=$1
d=gpurun_out/$tag; mkdir -p $d
export SEG_COMMIT=$(cat .commit 2>/dev/null)
for m in f32 bf16io; do
  bash tools/gpurun/roof.sh ${tag}_$m --math $m || exit 1
  python tools/queues.py gpurun_out/${tag}_$m/prof/run_kernel_trace.csv > gpurun_out/${tag}_$m/queues.txt || exit 1
done
timeout -k 10 400 python bench.py > $d/bench.json 2> $d/bench.err || { tail -5 $d/bench.err; exit 1; }
bash tools/gpurun/unet_cfg5.sh ${tag}_unet || exit 1
tail -c 400 $d/bench.json
