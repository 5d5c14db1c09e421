#!/bin/bash
# round 6: tests of the new kernels (upsample fold, weight-resident halo) + ADVICE fixes, the world-1 RCCL block,
# halo / igemm2 microbenchmarks (incl. DMA-off / MFMA-off builds), the fused2 Winograd diagnosis
t=${1:-r06d}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
: tests passed in the previous call

timeout -k 10 300 python tools/ig2bench.py --set unet --kernel halo --reps 10 > $d/halobench_unet.txt 2>&1 || { tail -5 $d/halobench_unet.txt; exit 1; }
timeout -k 10 300 python tools/ig2bench.py --set mnv2 --kernel halo --reps 10 > $d/halobench_mnv2.txt 2>&1 || { tail -5 $d/halobench_mnv2.txt; exit 1; }
cat $d/halobench_unet.txt $d/halobench_mnv2.txt
for v in base variants/ig2_nodma.so variants/ig2_nomfma.so; do
  echo "== $v"
  if [ $v = base ]; then timeout -k 10 300 python tools/ig2bench.py --set unet --kernel ig2 --reps 10; else SEG_LIB_PATH=$v timeout -k 10 300 python tools/ig2bench.py --set unet --kernel ig2 --reps 10; fi
  rc=$?; [ $rc -ne 0 ] && exit $rc
done > $d/ig2diag.txt 2>&1
cat $d/ig2diag.txt
SEG_LIB_PATH=variants/wf2.so timeout -k 10 600 python tools/wf2diag.py > $d/wf2diag.txt 2>&1
rc=$?; tail -25 $d/wf2diag.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-unet-block --no-infer-block > $d/bench.json 2> $d/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -5 $d/bench.err; exit $rc; }
python -c "import json; d=json.loads(open('$d/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['bf16io']['value']); print(json.dumps(d['multi_gpu'], indent=1))"
