set -o pipefail
d=gpurun_out/r04b4; mkdir -p $d
timeout -k 10 400 python -u -m pytest tests/test_gpu_infer.py tests/test_gpu_mbconv.py tests/test_gpu_splitk_ic.py -q --timeout 200 --timeout-method thread > $d/pytest.log 2>&1 || { tail -30 $d/pytest.log; exit 1; }
tail -2 $d/pytest.log
bash tools/gpurun/ab.sh r04b4 3 "--workload infer --frames 2000" base SEG_PLAN_B1=0 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $d/prof -o run --output-format csv -- python bench.py --workload infer --frames 50 --no-cpu-baseline > $d/prof.log 2>&1 || { tail -5 $d/prof.log; exit 1; }
python tools/trace_frame.py $(ls $d/prof/*/run_kernel_trace.csv $d/prof/run_kernel_trace.csv 2>/dev/null | head -1) > $d/frame.md
tail -1 $d/frame.md
