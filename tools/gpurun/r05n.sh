#!/bin/bash
# inference: the deadlock-free tile combine against round 4's unbounded spin (test-only build), interleaved; the
# combine / inference / op tests (hand-off path forced through seg_set_combine_spin)
t=${1:-r05n}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_infer.py tests/test_gpu_splitk_ic.py tests/test_gpu_mbconv.py tests/test_gpu_ops.py -k "not test_conv_wino_wgrad" -x -q --timeout 200 --timeout-method thread > $d/tests.log 2>&1 || { tail -5 $d/tests.log; exit 1; }
grep -E "passed|failed" $d/tests.log
for r in 1 2 3; do
  for v in base legacycomb; do
    if [ $v = base ]; then env=(); else env=(SEG_LIB_PATH=variants/$v.so); fi
    env "${env[@]}" timeout -k 10 200 python bench.py --workload infer --no-cpu-baseline > $d/b.json 2> $d/b.err || { tail -5 $d/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$d/b.json').read().strip().splitlines()[-1]); print('$r', '$v', d['value'], d.get('ms_per_step'))" | tee -a $d/ab.txt
  done
done
