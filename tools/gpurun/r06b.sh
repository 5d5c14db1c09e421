#!/bin/bash
# round 6: ADVICE-fix tests, the world-1 RCCL DataParallel block, igemm2 / halo diagnostics (DMA off / MFMA off builds)
t=${1:-r06b}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_ddp.py tests/test_gpu_infer.py tests/test_gpu_mbconv.py > $d/pytest.log 2>&1
rc=$?; tail -3 $d/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-unet-block --no-infer-block > $d/bench.json 2> $d/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -5 $d/bench.err; exit $rc; }
python -c "import json; d=json.loads(open('$d/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['bf16io']['value']); print(json.dumps(d['multi_gpu'], indent=1))"
for v in base variants/ig2_nodma.so variants/ig2_nomfma.so; do
  echo "== $v"
  if [ $v = base ]; then timeout -k 10 300 python tools/ig2bench.py --set unet --kernel all --reps 10; else SEG_LIB_PATH=$v timeout -k 10 300 python tools/ig2bench.py --set unet --kernel all --reps 10; fi
  rc=$?; [ $rc -ne 0 ] && exit $rc
done > $d/ig2bench.txt 2>&1
cat $d/ig2bench.txt
SEG_LIB_PATH=variants/wf2.so timeout -k 10 600 python tools/wf2diag.py > $d/wf2diag.txt 2>&1
rc=$?; cat $d/wf2diag.txt | tail -25; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in 1 0; do
    SEG_UPFOLD=$v timeout -k 10 300 python bench.py --workload infer --no-cpu-baseline > $d/inf.json 2>&1 || { tail -5 $d/inf.json; exit 1; }
    python -c "import json; d=json.loads(open('$d/inf.json').read().strip().splitlines()[-1]); print('$r UPFOLD=$v', d['value'], d['latency_ms'])" | tee -a $d/ab_upfold.txt
  done
done
