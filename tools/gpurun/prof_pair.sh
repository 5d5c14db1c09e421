#!/bin/bash
# roofline profile (kernel trace + PMC passes) of the f32 and bf16io bench configurations,
# plus the per-queue step breakdown: gpurun_out/<tag>_{f32,bf16io}/
set -o pipefail
tag=$1; shift
export SEG_COMMIT=$(cat .commit 2>/dev/null)
bash tools/gpurun/gpurun_roof.sh ${tag}_f32 "$@" || exit 1
python tools/queues.py gpurun_out/${tag}_f32/prof/run_kernel_trace.csv > gpurun_out/${tag}_f32/queues.txt || exit 1
bash tools/gpurun/gpurun_roof.sh ${tag}_bf16io --math bf16io "$@" || exit 1
python tools/queues.py gpurun_out/${tag}_bf16io/prof/run_kernel_trace.csv > gpurun_out/${tag}_bf16io/queues.txt || exit 1
head -30 gpurun_out/${tag}_bf16io/queues.txt
