#!/bin/bash
# PMC passes over the depthwise microbenchmark (tools/dwbench.py): gpurun_out/$1/<pass>/
export TMPDIR=/tmp
d=gpurun_out/$1; shift
mkdir -p $d
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d $d/p$i -o run --output-format csv -- python tools/dwbench.py "$@" > $d/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
