#!/bin/bash
# Round-5 final tree: -m gpu suite, smoke, the f32 roofline profile (PMC) and the default bench line.
t=${1:-r05q}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp SEG_COMMIT=$(cat .commit 2>/dev/null)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $d/pytest.log 2>&1 || { tail -15 $d/pytest.log; exit 1; }
tail -2 $d/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $d/smoke.log 2>&1 || { tail -5 $d/smoke.log; exit 1; }
tail -1 $d/smoke.log
bash tools/gpurun/roof.sh ${t}_f32 --math f32 || exit 1
python tools/queues.py gpurun_out/${t}_f32/prof/run_kernel_trace.csv > gpurun_out/${t}_f32/queues.txt || exit 1
timeout -k 10 400 python bench.py > $d/bench.json 2> $d/bench.err || { tail -5 $d/bench.err; exit 1; }
tail -c 300 $d/bench.json
