#!/bin/bash
# GPU tests, then an A/B of the current library against tmp_ab/libsegamd_old.so (f32 and bf16io)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu.log 2>&1
rc=$?; tail -n 15 gpurun_out/gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh tmp_ab/libsegamd_old.so || exit 1
bash tools/ab_lib.sh tmp_ab/libsegamd_old.so --math bf16io || exit 1
