#!/bin/bash
# fused Winograd timing experiments (SEG_WF_EXP variants: 1 no loads, 2 no transform, 4 no MFMAs, 3 = 1|2)
t=${1:-r05h}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/wfbench.py base > $d/wf.txt 2>&1 || { tail -5 $d/wf.txt; exit 1; }
for v in 1 2 3 4; do
  SEG_LIB_PATH=variants/wf$v.so timeout -k 10 120 python -u tools/wfbench.py exp$v >> $d/wf.txt 2>&1 || { tail -5 $d/wf.txt; exit 1; }
done
cat $d/wf.txt
