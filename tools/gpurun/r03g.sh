#!/bin/bash
# Round-3 pass g: the thin-K pointwise kernel (seg_conv_pw): its test first, the -m gpu suite
# and smoke with it on, a per-launch profile and an interleaved A/B against SEG_PW=0.
t=r03g
bash tools/gpurun/steps.sh $t \
  "pw|180|python -u -m pytest tests/test_gpu_pw.py -x -q --timeout 60 --timeout-method thread" \
  "pytest|500|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "tp_bf16io|300|SEG_OVERLAP=0 python tools/tapeprof.py --math bf16io --top 100 --csv gpurun_out/$t/tp_bf16io.csv" \
  "ab_bf16io|400|bash tools/gpurun/ab.sh ${t}_bf16io 2 '--math bf16io' base SEG_PW=0" \
  "ab_f32|400|bash tools/gpurun/ab.sh ${t}_f32 2 '--math f32' base SEG_PW=0"
