#!/bin/bash
# A/B of the engine's optional fusions on one box: img/s of bench.py (no timer) per flag set.
# usage: bash tools/ab_flags.sh [bench args]
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timer "${ARGS[@]}" > gpurun_out/ab.log 2>&1 || { echo "$label failed"; tail -3 gpurun_out/ab.log; exit 1; }
  echo "$label $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
}
ARGS=("$@")
for i in 1 2; do
  run base SEG_X=0
  run bnred SEG_BN_RED=1
  run bnb SEG_BNB=1
  run bnb+red SEG_BNB=1 SEG_BN_RED=1
  run pwfused SEG_PW_FUSED=1
done
