#!/bin/bash
# fused Winograd: op parity + per-shape timing
t=${1:-r05i}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
bash tools/gpurun/steps.sh $t \
  "tests|300|python -u -m pytest tests/test_gpu_ops.py -k wino -x -q --timeout 120 --timeout-method thread" || exit 1
grep -q passed $d/tests.log && ! grep -q failed $d/tests.log || exit 1
timeout -k 10 120 python -u tools/wfbench.py base > $d/wf.txt 2>&1 || { tail -5 $d/wf.txt; exit 1; }
cat $d/wf.txt
