#!/bin/bash
# img/s of bench.py (no timer) for each conv math on one box, interleaved twice.
for i in 1 2; do
  for m in "$@"; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timer --math $m > gpurun_out/abm.log 2>&1 || { echo "$m failed"; tail -3 gpurun_out/abm.log; exit 1; }
    echo "math=$m $(grep -o '"value": [0-9.]*' gpurun_out/abm.log)"
  done
done
