#!/bin/bash
# Per-launch profiles (tools/tapeprof.py, side stream off) of each variant (see ab.sh):
#   tape.sh <tag> "<tapeprof args, e.g. --math bf16io --top 60>" <variant>...
tag=$1; targs=$2; shift 2
d=gpurun_out/$tag; mkdir -p $d
for v in "$@"; do
  envs=(SEG_OVERLAP=0)
  for kv in $v; do
    case $kv in base) ;; lib=*) envs+=("SEG_LIB_PATH=${kv#lib=}") ;; *) envs+=("$kv") ;; esac
  done
  n=$(echo "$v" | tr ' /=' '___')
  env "${envs[@]}" timeout -k 10 300 python tools/tapeprof.py $targs > $d/tp_$n.txt 2>&1 || { echo "$v failed"; tail -5 $d/tp_$n.txt; exit 1; }
  head -12 $d/tp_$n.txt
done
