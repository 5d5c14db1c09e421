#!/bin/bash
# round 6: BatchNorm backward formed on load (bwx) -- kernel parity, model parity, step A/B, per-launch tape
t=${1:-r06j}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bwx.py > $d/pytest_bwx.log 2>&1
rc=$?; tail -3 $d/pytest_bwx.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $d/pytest_bwx.log | head -20; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_bf16io.py tests/test_gpu_bnout.py tests/test_gpu_tape.py tests/test_gpu_lazy_pw.py > $d/pytest_model.log 2>&1
rc=$?; tail -3 $d/pytest_model.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $d/pytest_model.log | head -20; exit $rc; }
bash tools/gpurun/ab.sh $t 2 "--math bf16io" base "SEG_BWX=0" "SEG_BWX_W=0" || exit 1
bash tools/gpurun/ab.sh $t 2 "--math f32" base "SEG_BWX=0" || exit 1
SEG_OVERLAP=0 timeout -k 10 300 python -u tools/tapeprof.py --math bf16io --steps 3 --top 400 --csv $d/tp_bf16io.csv > $d/tp_bf16io.txt 2>&1 || { tail -20 $d/tp_bf16io.txt; exit 1; }
head -40 $d/tp_bf16io.txt
