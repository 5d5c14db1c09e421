#!/bin/bash
# Run GPU steps in order; stop at the first crash/timeout (rc > 1), keep going on plain test failures.
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    ops)   run ops 600 python -m pytest tests/test_gpu_ops.py -q -m gpu ;;
    model) run model 900 python -m pytest tests/test_gpu_model.py -q -m gpu -x ;;
    gpu)   run gpu 1200 python -m pytest tests -q -m gpu ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 10 --warmup 3 ;;
    bf16)  run bf16 600 python -u -m pytest tests/test_gpu_bf16.py -q -m gpu -x -s --timeout 300 --timeout-method thread ;;
    benchbf) run benchbf 600 python bench.py --steps 10 --warmup 3 --math bf16 --no-cpu-baseline ;;
    unetbf) run unetbf 600 python bench.py --model UNet --height 512 --width 1024 --batch 8 --steps 3 --warmup 2 --math bf16 --no-cpu-baseline ;;
    inferg) run inferg 600 python -u -m pytest tests/test_gpu_infer.py -q -m gpu -x -s --timeout 300 --timeout-method thread ;;
    infer32) run infer32 600 python bench.py --workload infer --frames 300 --math f32 --no-cpu-baseline ;;
    bf16io) run bf16io 600 python -u -m pytest tests/test_gpu_bf16io.py -q -m gpu -x --timeout 120 --timeout-method thread ;;
    benchio) run benchio 600 python bench.py --steps 10 --warmup 3 --math bf16io --no-cpu-baseline ;;
    graph) run graph 600 python -u -m pytest tests/test_gpu_graph.py -q -m gpu -x --timeout 300 --timeout-method thread ;;
    benchq) run benchq 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    unet) run unet 600 python bench.py --model UNet --height 512 --width 1024 --batch 8 --steps 3 --warmup 2 ;;
    infer) run infer 600 python bench.py --workload infer --frames 300 --cpu-seconds 8 ;;
  esac
done
