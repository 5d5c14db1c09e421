#!/bin/bash
# fused Winograd: op parity (both forms) and per-shape timing against the direct / two-launch Winograd kernels
t=${1:-r05g}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
bash tools/gpurun/steps.sh $t \
  "tests|300|python -u -m pytest tests/test_gpu_ops.py -k wino -x -q --timeout 120 --timeout-method thread" || exit 1
grep -q passed $d/tests.log && ! grep -q failed $d/tests.log || exit 1
timeout -k 10 300 python -u tools/winobench.py > $d/winobench.txt 2>&1 || { tail -5 $d/winobench.txt; exit 1; }
cat $d/winobench.txt
