#!/bin/bash
# bf16 packed weights: bitwise tests, bf16io model parity, interleaved A/B (MobileNetV2UNet and UNet 512x1024)
tag=$1
d=gpurun_out/$tag; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests/test_gpu_w16.py tests/test_gpu_bf16io.py tests/test_gpu_unet_cfg5.py tests/test_gpu_lazy_pw.py -x -q --timeout 300 --timeout-method thread > $d/pytest.log 2>&1
rc=$?; tail -3 $d/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpurun/ab.sh $tag bf16io 3 "SEG_W16=0" "SEG_W16=1" || exit 1
for r in 1 2; do for cfg in "SEG_W16=0" "SEG_W16=1"; do
  env $cfg timeout -k 10 200 python bench.py --model UNet --height 512 --width 1024 --batch 8 --math bf16io --steps 10 --warmup 3 --no-cpu-baseline > $d/u.json 2> $d/u.err || { echo "UNet $cfg FAILED"; tail -5 $d/u.err; exit 1; }
  python -c "import json; d=json.loads(open('$d/u.json').read().strip().splitlines()[-1]); print('unet bf16io', '$cfg', d['value'], d['ms_per_step'])"
done; done
SEG_OVERLAP=0 timeout -k 10 200 python tools/tapeprof.py --math bf16io --top 60 > $d/tp_bf16io_noov.txt 2>&1 || exit 1
head -12 $d/tp_bf16io_noov.txt
