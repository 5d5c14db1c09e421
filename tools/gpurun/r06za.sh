#!/bin/bash
# round 6: MobileNetV2UNet f32 contention table on the wino_wgrad16 + one-row partials tree (side stream on / off)
t=${1:-r06za}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp
A="--steps 4 --warmup 2 --no-cpu-baseline --no-timer --no-bf16io-block --no-infer-block --no-unet-block --no-dp1-block"
timeout -k 10 300 rocprofv3 --kernel-trace -d $d/on -o run --output-format csv -- python bench.py $A > $d/on.log 2>&1 || { tail -5 $d/on.log; exit 1; }
SEG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $d/off -o run --output-format csv -- python bench.py $A > $d/off.log 2>&1 || { tail -5 $d/off.log; exit 1; }
python tools/contention.py $(ls $d/on/run_kernel_trace.csv $d/on/*/run_kernel_trace.csv 2>/dev/null | head -1) $(ls $d/off/run_kernel_trace.csv $d/off/*/run_kernel_trace.csv 2>/dev/null | head -1) --md $d/contention_f32.md > /dev/null || exit 1
head -60 $d/contention_f32.md
