#!/bin/bash
# Round-3 re-entry pass: -m gpu suite, smoke, default bench line, per-launch profiles,
# the model suites again with SEG_BX=1 (1x1 dgrads forming dY on load).
t=r03a
bash tools/gpurun/steps.sh $t \
  "pytest|600|python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread" \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py --steps 20 --warmup 5" \
  "pytest_bx|400|SEG_BX=1 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bf16io.py tests/test_gpu_tape.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread" \
  "tp_bf16io|300|SEG_OVERLAP=0 python tools/tapeprof.py --math bf16io --top 100 --csv gpurun_out/$t/tp_bf16io.csv" \
  "tp_bf16io_bx|300|SEG_OVERLAP=0 SEG_BX=1 python tools/tapeprof.py --math bf16io --top 100 --csv gpurun_out/$t/tp_bf16io_bx.csv" \
  "tp_f32|300|SEG_OVERLAP=0 python tools/tapeprof.py --math f32 --top 100 --csv gpurun_out/$t/tp_f32.csv" \
  "tp_bf16io_noig2|300|SEG_OVERLAP=0 SEG_IGEMM2=0 python tools/tapeprof.py --math bf16io --top 100 --csv gpurun_out/$t/tp_bf16io_noig2.csv" \
  "ig2bench|200|python tools/ig2bench.py"
