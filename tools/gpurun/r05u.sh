#!/bin/bash
# BN channel reductions over up to 512 row blocks (256-thread blocks: the thread count of the old 512 x 256) A/B,
# with the BN / bf16io op tests on the variant
t=${1:-r05u}
d=gpurun_out/$t; mkdir -p $d
SEG_LIB_PATH=variants/maxblk512.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16io.py tests/test_gpu_ops.py -k "bn or stats or backward or colsum" -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1 || { tail -8 $d/tests.log; exit 1; }
grep -E "passed|failed" $d/tests.log
bash tools/gpurun/ab.sh ${t} 2 "--math bf16io" base "lib=variants/maxblk512.so" || exit 1
bash tools/gpurun/ab.sh ${t} 2 "--math f32" base "lib=variants/maxblk512.so" || exit 1
cat gpurun_out/${t}/ab.txt
