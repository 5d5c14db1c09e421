#!/bin/bash
# interleaved A/B of library builds on MobileNetV2UNet bf16io and UNet 512x1024 bs=8 bf16io: libab2.sh <tag> <rounds>
tag=$1; rounds=$2
d=gpurun_out/$tag; mkdir -p $d
for r in $(seq $rounds); do
  for lib in team02-objectdetection_amd/seg_amd/_lib/libsegamd.so variants/*.so; do
    SEG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 30 --warmup 5 --math bf16io --no-cpu-baseline > $d/b.json 2> $d/b.err || { echo "$lib FAILED"; tail -5 $d/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$d/b.json').read().strip().splitlines()[-1]); print('mnv2', '$(basename $lib .so)', d['value'], d['ms_per_step'])"
    SEG_LIB_PATH=$lib timeout -k 10 200 python bench.py --model UNet --height 512 --width 1024 --batch 8 --math bf16io --steps 10 --warmup 3 --no-cpu-baseline > $d/u.json 2> $d/u.err || { echo "$lib UNet FAILED"; tail -5 $d/u.err; exit 1; }
    python -c "import json; d=json.loads(open('$d/u.json').read().strip().splitlines()[-1]); print('unet', '$(basename $lib .so)', d['value'], d['ms_per_step'])"
  done
done
