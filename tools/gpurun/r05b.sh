#!/bin/bash
# Round 5: -m gpu suite, then the roofline profiles (kernel trace + FETCH / WRITE / MFMA PMC passes) of both maths
# with the side stream on, and a kernel trace with it off (tools/contention.py).
t=${1:-r05b}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp SEG_COMMIT=$(cat .commit 2>/dev/null)
bash tools/gpurun/steps.sh $t \
  "pytest|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" || exit 1
for m in bf16io f32; do
  bash tools/gpurun/roof.sh ${t}_$m --math $m || exit 1
  python tools/queues.py gpurun_out/${t}_$m/prof/run_kernel_trace.csv > gpurun_out/${t}_$m/queues.txt || exit 1
  SEG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${t}_$m/alone -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-timer --no-bf16io-block --no-infer-block --no-unet-block --math $m > gpurun_out/${t}_$m/alone.log 2>&1 || exit 1
  python tools/contention.py gpurun_out/${t}_$m/prof/run_kernel_trace.csv gpurun_out/${t}_$m/alone/run_kernel_trace.csv --md gpurun_out/${t}_$m/contention.md > /dev/null || exit 1
  echo "== $m profiled"
done
