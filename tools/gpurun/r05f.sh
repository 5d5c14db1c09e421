#!/bin/bash
# tile-combine protocol check: split-K in-launch combine, fused MBConv, two concurrent predictors; inference bench
t=${1:-r05f}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp SEG_COMMIT=$(cat .commit 2>/dev/null)
bash tools/gpurun/steps.sh $t \
  "tests|400|python -u -m pytest tests/test_gpu_infer.py tests/test_gpu_splitk_ic.py tests/test_gpu_mbconv.py -x -q --timeout 120 --timeout-method thread" || exit 1
grep -q passed $d/tests.log && ! grep -q failed $d/tests.log || exit 1
timeout -k 10 300 python bench.py --workload infer > $d/infer.json 2> $d/infer.err || { tail -5 $d/infer.err; exit 1; }
tail -c 400 $d/infer.json
