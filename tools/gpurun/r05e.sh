#!/bin/bash
# BNOUT bf16io parity cases + concurrent predictors, configs[4] (UNet 8x512x1024 bf16io) roofline profile with PMC,
# and the default bench line (f32 headline, nested bf16io / UNet / inference blocks, BN-backward rooflines)
t=${1:-r05e}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp SEG_COMMIT=$(cat .commit 2>/dev/null)
bash tools/gpurun/steps.sh $t \
  "parity|400|python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_infer.py -k 'model_bf16 or two_predictors' -x -q -s --timeout 200 --timeout-method thread" || exit 1
grep -q passed $d/parity.log && ! grep -q failed $d/parity.log || exit 1
ROOF_MODEL=UNet bash tools/gpurun/roof.sh ${t}_unet --math bf16io --model UNet --height 512 --width 1024 --batch 8 || exit 1
python tools/queues.py gpurun_out/${t}_unet/prof/run_kernel_trace.csv > gpurun_out/${t}_unet/queues.txt || exit 1
timeout -k 10 400 python bench.py > $d/bench.json 2> $d/bench.err || { tail -5 $d/bench.err; exit 1; }
tail -c 600 $d/bench.json
