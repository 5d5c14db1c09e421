#!/bin/bash
# two-waves-per-SIMD fused Winograd: op parity, per-shape timing (wfbench: fused2 vs fused1; winobench: vs direct /
# halo / two-launch on both models' shapes)
t=${1:-r05r}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "wino" -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1 || { tail -8 $d/tests.log; exit 1; }
grep -E "passed|failed" $d/tests.log
timeout -k 10 120 python -u tools/wfbench.py fused2 > $d/wf.txt 2>&1 || { tail -5 $d/wf.txt; exit 1; }
SEG_LIB_PATH=variants/wf1.so timeout -k 10 120 python -u tools/wfbench.py fused1 >> $d/wf.txt 2>&1 || { tail -5 $d/wf.txt; exit 1; }
cat $d/wf.txt
timeout -k 10 300 python -u tools/winobench.py > $d/winobench.txt 2>&1 || { tail -5 $d/winobench.txt; exit 1; }
WINOBENCH=unet timeout -k 10 400 python -u tools/winobench.py > $d/winobench_unet.txt 2>&1 || { tail -5 $d/winobench_unet.txt; exit 1; }
grep -E "fwd|dgrad" $d/winobench.txt | grep -v halo
