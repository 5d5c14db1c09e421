#!/bin/bash
# bf16io roofline profile (kernel trace + FETCH / WRITE / MFMA PMC) and contention table at the final tree
t=${1:-r05w}
export TMPDIR=/tmp SEG_COMMIT=$(cat .commit 2>/dev/null)
m=bf16io
bash tools/gpurun/roof.sh ${t}_$m --math $m || exit 1
python tools/queues.py gpurun_out/${t}_$m/prof/run_kernel_trace.csv > gpurun_out/${t}_$m/queues.txt || exit 1
SEG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${t}_$m/alone -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-timer --no-bf16io-block --no-infer-block --no-unet-block --no-dp1-block --math $m > gpurun_out/${t}_$m/alone.log 2>&1 || exit 1
python tools/contention.py gpurun_out/${t}_$m/prof/run_kernel_trace.csv gpurun_out/${t}_$m/alone/run_kernel_trace.csv --md gpurun_out/${t}_$m/contention.md > /dev/null || exit 1
head -12 gpurun_out/${t}_$m/${t}_$m.md
