#!/bin/bash
# End-of-round evidence, part 3: the GPU suite + smoke at HEAD and one inference frame's kernel trace.
set -o pipefail
tag=$1
d=gpurun_out/$tag; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $d/pytest.log 2>&1 || { tail -30 $d/pytest.log; exit 1; }
tail -2 $d/pytest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > $d/smoke.log 2>&1 || { tail -5 $d/smoke.log; exit 1; }
tail -1 $d/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $d/prof -o run --output-format csv -- python bench.py --workload infer --frames 50 --no-cpu-baseline > $d/prof.log 2>&1 || { tail -5 $d/prof.log; exit 1; }
python tools/trace_frame.py $(ls $d/prof/*/run_kernel_trace.csv $d/prof/run_kernel_trace.csv 2>/dev/null | head -1) > $d/frame.md
tail -1 $d/frame.md
