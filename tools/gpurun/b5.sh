set -o pipefail
d=gpurun_out/r04b5; mkdir -p $d
timeout -k 10 400 python -u -m pytest tests/test_gpu_infer.py tests/test_gpu_mbconv.py -q --timeout 200 --timeout-method thread > $d/pytest.log 2>&1 || { tail -30 $d/pytest.log; exit 1; }
tail -2 $d/pytest.log
bash tools/gpurun/ab.sh r04b5 3 "--workload infer --frames 2000" base SEG_STEM_PRE=0 || exit 1
