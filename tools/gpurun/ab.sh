#!/bin/bash
# Interleaved A/B of variants on one box -- the one A/B script.
#   ab.sh <tag> <rounds> "<bench.py args>" <variant>...
# A variant is a space-separated list of ENV=value settings and/or lib=<path to a
# libsegamd.so build> (SEG_LIB_PATH); "base" is the tree as it is.  Each round runs every
# variant once (same order), one bench line each: gpurun_out/<tag>/ab.txt.
#   e.g. ab.sh w16 3 "--math bf16io" base "SEG_W16=0" "lib=variants/old.so"
tag=$1; rounds=$2; bargs=$3; shift 3
d=gpurun_out/$tag; mkdir -p $d
for r in $(seq $rounds); do
  for v in "$@"; do
    envs=()
    for kv in $v; do
      case $kv in
        base) ;;
        lib=*) envs+=("SEG_LIB_PATH=${kv#lib=}") ;;
        *) envs+=("$kv") ;;
      esac
    done
    env "${envs[@]}" timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-bf16io-block --no-infer-block --no-unet-block --no-dp1-block $bargs > $d/b.json 2> $d/b.err || { echo "$v FAILED"; tail -5 $d/b.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$d/b.json').read().strip().splitlines()[-1]); print('$r', '$v', '$bargs', d['value'], d['ms_per_step'])" | tee -a $d/ab.txt
  done
done
