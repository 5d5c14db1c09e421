#!/bin/bash
# Evidence pass (usage: evidence.sh <tag>): -m gpu suite + smoke, then final.sh (roofline profiles of f32 / bf16io:
# kernel trace + FETCH / WRITE / MFMA-busy PMC passes + per-queue breakdown, the default bench
# line, configs[4] lines).
t=${1:-evidence}
bash tools/gpurun/steps.sh $t \
  "pytest|400|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" || exit 1
grep -q "passed" gpurun_out/$t/pytest.log && ! grep -q "failed" gpurun_out/$t/pytest.log || exit 1
bash tools/gpurun/final.sh $t
