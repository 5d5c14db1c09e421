#!/bin/bash
# prefetch depth: 16-bit GEMM tests, then interleaved A/B of library builds (bench value)
tag=$1; shift
d=gpurun_out/$tag; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_bf16io.py -x -q --timeout 300 --timeout-method thread > $d/pytest.log 2>&1
rc=$?; tail -3 $d/pytest.log; [ $rc -ne 0 ] && exit $rc
for math in "$@"; do
 for r in 1 2 3; do
  for lib in team02-objectdetection_amd/seg_amd/_lib/libsegamd.so variants/*.so; do
    SEG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 30 --warmup 5 --math $math --no-cpu-baseline > $d/b.json 2> $d/b.err || { echo "$lib FAILED"; tail -5 $d/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$d/b.json').read().strip().splitlines()[-1]); print('$math', '$lib', d['value'], d['ms_per_step'])"
  done
 done
done
