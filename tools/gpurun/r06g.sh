#!/bin/bash
# round 6: igemm2 K-step 32 form (tests, per-launch, step A/B) and the per-level upsample fold (batch-1 inference)
t=${1:-r06g}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_igemm2.py tests/test_gpu_mbconv.py > $d/pytest.log 2>&1
rc=$?; tail -2 $d/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $d/pytest.log | head; exit $rc; }
timeout -k 10 300 python tools/ig2bench.py --set unet --kernel ig2 --reps 10 > $d/ig2kb_unet.txt 2>&1 || { tail -5 $d/ig2kb_unet.txt; exit 1; }
timeout -k 10 300 python tools/ig2bench.py --set mnv2 --kernel ig2 --reps 20 > $d/ig2kb_mnv2.txt 2>&1 || { tail -5 $d/ig2kb_mnv2.txt; exit 1; }
cat $d/ig2kb_unet.txt $d/ig2kb_mnv2.txt
bash tools/gpurun/ab.sh ${t} 2 "--model UNet --height 512 --width 1024 --batch 8 --math bf16io" base "SEG_IG2_KB=32" || exit 1
bash tools/gpurun/ab.sh ${t} 2 "--math bf16io" base "SEG_IG2_KB=32" || exit 1
for r in 1 2; do
  for v in 0 1 2 4 8; do
    SEG_UPFOLD=$v timeout -k 10 300 python bench.py --workload infer --no-cpu-baseline > $d/inf.json 2>&1 || { tail -5 $d/inf.json; exit 1; }
    python -c "import json; d=json.loads(open('$d/inf.json').read().strip().splitlines()[-1]); print('$r UPFOLD=$v', d['value'], d['latency_ms'])" | tee -a $d/ab_upfold.txt
  done
done
cat $d/ab.txt
