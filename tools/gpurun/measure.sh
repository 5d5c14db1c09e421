#!/bin/bash
# regression suite + both bench configurations + the no-overlap per-launch profile of bf16io
tag=$1
bash tools/gpurun/check.sh $tag || exit 1
d=gpurun_out/$tag
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --math bf16io --no-cpu-baseline > $d/bf16io.json 2>&1 || exit 1
SEG_OVERLAP=0 timeout -k 10 200 python tools/tapeprof.py --math bf16io --top 40 > $d/tp_bf16io_noov.txt 2>&1 || exit 1
python - <<PY
import json
for f in ["$d/bench.json", "$d/bf16io.json"]:
    d = json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"])
PY
head -20 $d/tp_bf16io_noov.txt
