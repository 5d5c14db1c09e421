#!/bin/bash
# regression suite + both bench configurations + per-launch profiles (f32 and bf16io, in-step and
# without the side stream) + a kernel-trace of f32 for the per-queue busy / idle breakdown
tag=$1
bash tools/gpurun/check.sh $tag || exit 1
d=gpurun_out/$tag
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --math bf16io --no-cpu-baseline > $d/bf16io.json 2>&1 || exit 1
timeout -k 10 200 python tools/tapeprof.py --math f32 --top 60 > $d/tp_f32.txt 2>&1 || exit 1
SEG_OVERLAP=0 timeout -k 10 200 python tools/tapeprof.py --math f32 --top 60 > $d/tp_f32_noov.txt 2>&1 || exit 1
SEG_OVERLAP=0 timeout -k 10 200 python tools/tapeprof.py --math bf16io --top 60 > $d/tp_bf16io_noov.txt 2>&1 || exit 1
bash tools/gpurun/gpurun_prof.sh ${tag}_f32prof || exit 1
python tools/queues.py gpurun_out/${tag}_f32prof/run_kernel_trace.csv > $d/queues_f32.txt || exit 1
python - <<PY
import json
for f in ["$d/bench.json", "$d/bf16io.json"]:
    d = json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"])
PY
cat $d/queues_f32.txt
