#!/bin/bash
# SQ / TCC counter passes (one rocprofv3 --pmc run each, kernel trace only) over a short bench run,
# side stream off so each dispatch's counters are its own; table: gpurun_out/$1/sq.md
#   usage: bash tools/gpurun/sq.sh <name> [bench.py args]
export TMPDIR=/tmp
name=$1; shift
d=gpurun_out/$name; mkdir -p $d
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_LDS" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  SEG_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d $d/p$i -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timer --no-bf16io-block --no-infer-block --no-unet-block --no-dp1-block "$@" > $d/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $d/p$i.log; exit $rc; }
done
python tools/sq_report.py $d/sq.md $d/p1 $d/p2 $d/p3 > /dev/null && head -30 $d/sq.md
