#!/bin/bash
# upsample-backward kernel shape under side-stream contention: quad (default) vs plain vs quad with 2 rows in flight
t=${1:-r05l}
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_ops.py -k "upsample or up2" -x -q --timeout 120 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1 || { tail -5 gpurun_out/${t}_tests.log; exit 1; }
SEG_LIB_PATH=variants/quadu2.so timeout -k 10 120 python -u -m pytest tests/test_gpu_ops.py -k "upsample or up2" -x -q --timeout 120 --timeout-method thread >> gpurun_out/${t}_tests.log 2>&1 || { tail -5 gpurun_out/${t}_tests.log; exit 1; }
bash tools/gpurun/ab.sh ${t}_ab 2 "--math f32" base "lib=variants/noquad.so" "lib=variants/quadu2.so" || exit 1
bash tools/gpurun/ab.sh ${t}_ab 2 "--math bf16io" base "lib=variants/noquad.so" "lib=variants/quadu2.so" || exit 1
grep -E "passed|failed" gpurun_out/${t}_tests.log
