#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run into gpurun_out/$1
export TMPDIR=/tmp
d=gpurun_out/$1; shift
mkdir -p $d
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-timer "$@" > $d/bench.log 2>&1
rc=$?; echo "prof rc=$rc"; grep metric $d/bench.log | cut -c1-200; exit $rc
