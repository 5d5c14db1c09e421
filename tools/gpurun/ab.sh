#!/bin/bash
# Interleaved A/B of engine env knobs on one box: ab.sh <tag> <math> <rounds> "ENV=a" "ENV=b" ...
tag=$1; math=$2; rounds=$3; shift 3
d=gpurun_out/$tag; mkdir -p $d
for r in $(seq $rounds); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 120 python bench.py --steps 30 --warmup 5 --math $math --no-cpu-baseline > $d/b.json 2> $d/b.err || { echo "$cfg FAILED"; tail -5 $d/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$d/b.json').read().strip().splitlines()[-1]); print('$math', '$cfg', d['value'], d['ms_per_step'])"
  done
done
