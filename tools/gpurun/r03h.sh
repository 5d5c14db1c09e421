#!/bin/bash
# Round-3 pass h: thin-K pointwise convs restricted to >= 256k-row layers: interleaved A/B and
# kernel traces of the real (overlapped) bf16io step with and without them.
t=r03h
export TMPDIR=/tmp
bash tools/gpurun/steps.sh $t \
  "ab_bf16io|500|bash tools/gpurun/ab.sh ${t}_bf16io 3 '--math bf16io' base SEG_PW=0" \
  "ab_f32|400|bash tools/gpurun/ab.sh ${t}_f32 2 '--math f32' base SEG_PW=0" \
  "trace_pw|200|rocprofv3 --kernel-trace --stats -d gpurun_out/$t/pw -o run --output-format csv -- python bench.py --math bf16io --steps 5 --warmup 2 --no-cpu-baseline --no-timer --no-bf16io-block --no-infer-block" \
  "trace_nopw|200|SEG_PW=0 rocprofv3 --kernel-trace --stats -d gpurun_out/$t/nopw -o run --output-format csv -- python bench.py --math bf16io --steps 5 --warmup 2 --no-cpu-baseline --no-timer --no-bf16io-block --no-infer-block"
