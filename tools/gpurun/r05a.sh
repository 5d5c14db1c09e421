#!/bin/bash
# Round 5 first call: the -m gpu suite + smoke at HEAD, then per-launch profiles (side stream off) of both maths
# for the BN-layer budget (tools/bn_layers.py).
t=${1:-r05a}
d=gpurun_out/$t; mkdir -p $d
bash tools/gpurun/steps.sh $t \
  "pytest|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "tp_bf16io|300|SEG_OVERLAP=0 python tools/tapeprof.py --math bf16io --top 80 --csv $d/tp_bf16io.csv" \
  "tp_f32|300|SEG_OVERLAP=0 python tools/tapeprof.py --math f32 --top 80 --csv $d/tp_f32.csv" || exit 1
