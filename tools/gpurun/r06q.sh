#!/bin/bash
# round 6: the decoder's weight gradients deferred to the encoder's backward (bf16io default) -- tests, A/B
t=${1:-r06q}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf16io.py tests/test_gpu_ddp.py tests/test_gpu_ddp_ranks.py tests/test_gpu_tape.py tests/test_gpu_unet_cfg5.py > $d/pytest.log 2>&1
rc=$?; tail -2 $d/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $d/pytest.log | head -20; exit $rc; }
bash tools/gpurun/ab.sh $t 2 "--math bf16io" base "SEG_DEFER_DECODER=0" || exit 1
bash tools/gpurun/ab.sh $t 2 "--model UNet --height 512 --width 1024 --batch 8 --math bf16io" base "SEG_DEFER_DECODER=0" || exit 1
cat $d/ab.txt
