#!/bin/bash
# End-of-round evidence, part 1 (final.sh split to fit one gpurun call): roofline profiles of f32 and bf16io.
set -o pipefail
tag=$1
export SEG_COMMIT=$(cat .commit 2>/dev/null)
for m in f32 bf16io; do
  bash tools/gpurun/roof.sh ${tag}_$m --math $m || exit 1
  python tools/queues.py gpurun_out/${tag}_$m/prof/run_kernel_trace.csv > gpurun_out/${tag}_$m/queues.txt || exit 1
done
