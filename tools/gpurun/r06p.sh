#!/bin/bash
# round 6: decoder weight gradients deferred until the backward reaches the encoder (SEG_WGRAD_DEFER=from:at)
t=${1:-r06p}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
SEG_WGRAD_DEFER=52:51 SEG_WGRAD_TAIL=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_tape.py tests/test_gpu_ddp.py > $d/pytest.log 2>&1
rc=$?; tail -2 $d/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $d/pytest.log | head -20; exit $rc; }
bash tools/gpurun/ab.sh $t 2 "--math f32" base "SEG_WGRAD_DEFER=52:51" "SEG_WGRAD_DEFER=52:40" "SEG_WGRAD_TAIL=4" "SEG_WGRAD_TAIL=10" || exit 1
bash tools/gpurun/ab.sh $t 2 "--math bf16io" base "SEG_WGRAD_DEFER=52:51" "SEG_WGRAD_DEFER=52:40" "SEG_WGRAD_TAIL=4" "SEG_WGRAD_TAIL=10" || exit 1
for v in "" "52:51"; do
  SEG_WGRAD_DEFER=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-bf16io-block --no-infer-block --no-unet-block --no-dp1-block > $d/loss_$v.json 2>/dev/null
  python -c "import json; d=json.loads(open('$d/loss_$v.json').read().strip().splitlines()[-1]); print('defer=$v final_loss', repr(d['final_loss']))" | tee -a $d/ab.txt
done
cat $d/ab.txt
