#!/bin/bash
# round 6 (second session): per-launch tape profiles (which kernel consumes each BN layer's dY), bf16io and f32
t=${1:-r06i}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
for m in bf16io f32; do
  SEG_OVERLAP=0 timeout -k 10 300 python -u tools/tapeprof.py --math $m --steps 3 --top 400 --csv $d/tp_$m.csv > $d/tp_$m.txt 2>&1 \
    || { tail -20 $d/tp_$m.txt; exit 1; }
done
head -30 $d/tp_bf16io.txt
