#!/bin/bash
# GPU tests, then bench with seg_amd.Adam vs torch.optim.Adam on one box (f32, bf16io)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu.log 2>&1
rc=$?; tail -n 15 gpurun_out/gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for math in f32 bf16io; do
    for o in seg torch; do
      timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timer --math $math --optimizer $o > gpurun_out/abo.log 2>&1 || { echo "failed"; tail -5 gpurun_out/abo.log; exit 1; }
      echo "$math $o $(grep -o '"value": [0-9.]*' gpurun_out/abo.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/abo.log)"
    done
  done
done
