#!/bin/bash
# interleaved A/B of the default library against every variants/*.so: libab.sh <tag> <rounds> <math>...
tag=$1; rounds=$2; shift 2
d=gpurun_out/$tag; mkdir -p $d
for math in "$@"; do
 for r in $(seq $rounds); do
  for lib in team02-objectdetection_amd/seg_amd/_lib/libsegamd.so variants/*.so; do
    SEG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 30 --warmup 5 --math $math --no-cpu-baseline > $d/b.json 2> $d/b.err || { echo "$lib FAILED"; tail -5 $d/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$d/b.json').read().strip().splitlines()[-1]); print('$math', '$(basename $lib .so)', d['value'], d['ms_per_step'])"
  done
 done
done
