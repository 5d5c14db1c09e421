#!/bin/bash
# Kernel-trace/stats profile + FETCH_SIZE / WRITE_SIZE PMC passes of a short bench run,
# then the roofline summary in gpurun_out/$1/$1.{md,json} (copy it into profiles/ afterwards).
# usage: bash roof.sh <name> [extra bench.py args, e.g. --math bf16]
set -o pipefail
export TMPDIR=/tmp
name=$1; shift
d=gpurun_out/$name
mkdir -p $d
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d/prof -o run --output-format csv -- python bench.py --steps 7 --warmup 2 --no-cpu-baseline --no-timer --no-bf16io-block --no-infer-block --no-unet-block --no-dp1-block "$@" > $d/prof.log 2>&1 || { echo "prof failed"; tail -5 $d/prof.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d $d/pmc/$c -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timer --no-bf16io-block --no-infer-block --no-unet-block --no-dp1-block "$@" > $d/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $d/pmc_$c.log; exit 1; }
done
# matrix-core activity: MFMA-busy cycles (all SIMDs) against the GPU-active clock (sum over the 8 XCDs)
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $d/pmc/MFMA -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timer --no-bf16io-block --no-infer-block --no-unet-block --no-dp1-block "$@" > $d/pmc_MFMA.log 2>&1 || { echo "pmc MFMA failed"; tail -5 $d/pmc_MFMA.log; exit 1; }
python tools/roofline_report.py $d/prof $d/pmc 9 $d/$name ${ROOF_MODEL:-MobileNetV2UNet}
