#!/bin/bash
# round 6 A/Bs: weight-resident halo on/off (UNet configs[4] + MobileNetV2UNet bf16io, f32), upsample fold on/off (infer)
t=${1:-r06e}
d=gpurun_out/$t; mkdir -p $d
bash tools/gpurun/ab.sh ${t} 2 "--model UNet --height 512 --width 1024 --batch 8 --math bf16io" base "SEG_HALO_WR=0" || exit 1
bash tools/gpurun/ab.sh ${t} 2 "--math bf16io" base "SEG_HALO_WR=0" || exit 1
bash tools/gpurun/ab.sh ${t} 2 "--math f32" base "SEG_HALO_WR=0" || exit 1
for r in 1 2; do
  for v in 1 0; do
    SEG_UPFOLD=$v timeout -k 10 300 python bench.py --workload infer --no-cpu-baseline > $d/inf.json 2>&1 || { tail -5 $d/inf.json; exit 1; }
    python -c "import json; d=json.loads(open('$d/inf.json').read().strip().splitlines()[-1]); print('$r UPFOLD=$v', d['value'], d['latency_ms'])" | tee -a $d/ab_upfold.txt
  done
done
cat $d/ab.txt
