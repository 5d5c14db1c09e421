#!/bin/bash
# PMC passes (one counter group per pass) over a short bench run: gpurun_out/$1/{fetch,write}
export TMPDIR=/tmp
d=gpurun_out/$1; shift
mkdir -p $d
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -d $d/$c -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timer "$@" > $d/$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
