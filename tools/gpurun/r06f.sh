#!/bin/bash
# round 6: fused2 root cause with max-pool choices matched; DDP stops at bucket completion; slice test; upfold A/B
t=${1:-r06f}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_unet_cfg5.py tests/test_gpu_ddp.py tests/test_gpu_ddp_ranks.py tests/test_gpu_halo_wr.py > $d/pytest.log 2>&1
rc=$?; grep -E "worst of budget|passed|failed" $d/pytest.log | tail -5; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $d/pytest.log | head; exit $rc; }
SEG_LIB_PATH=variants/wf2.so timeout -k 10 600 python tools/wf2diag.py > $d/wf2diag.txt 2>&1
rc=$?; tail -6 $d/wf2diag.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-unet-block --no-infer-block --no-bf16io-block > $d/bench.json 2> $d/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -5 $d/bench.err; exit $rc; }
python -c "import json; d=json.loads(open('$d/bench.json').read().strip().splitlines()[-1]); print(d['value']); print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != 'note'} for k, v in d['multi_gpu']['world1_rccl'].items()}))"
bash tools/gpurun/ab.sh ${t} 2 "--model UNet --height 512 --width 1024 --batch 8 --math bf16io" base "SEG_HALO_WR=1" || exit 1
for r in 1 2; do
  for v in 1 0; do
    SEG_UPFOLD=$v timeout -k 10 300 python bench.py --workload infer --no-cpu-baseline > $d/inf.json 2>&1 || { tail -5 $d/inf.json; exit 1; }
    python -c "import json; d=json.loads(open('$d/inf.json').read().strip().splitlines()[-1]); print('$r UPFOLD=$v', d['value'], d['latency_ms'])" | tee -a $d/ab_upfold.txt
  done
done
