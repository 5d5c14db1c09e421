#!/bin/bash
# fused head + mask: inference tests, then frame time against the two launches (interleaved, one process)
t=${1:-r05p}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mbconv.py tests/test_gpu_infer.py -x -q --timeout 200 --timeout-method thread > $d/tests.log 2>&1 || { tail -8 $d/tests.log; exit 1; }
grep -E "passed|failed" $d/tests.log
timeout -k 10 300 python -u tools/headbench.py 4 500 > $d/headbench.txt 2>&1 || { tail -5 $d/headbench.txt; exit 1; }
cat $d/headbench.txt
timeout -k 10 200 python bench.py --workload infer --no-cpu-baseline > $d/infer.json 2> $d/infer.err || { tail -5 $d/infer.err; exit 1; }
python -c "import json; d=json.loads(open('$d/infer.json').read().strip().splitlines()[-1]); print('bench infer', d['value'])"
