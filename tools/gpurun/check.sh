#!/bin/bash
# GPU regression pass: the -m gpu suite, smoke, and one default bench line.
# usage: bash tools/gpurun/check.sh <tag> [extra pytest args]
tag=$1; shift
d=gpurun_out/$tag; mkdir -p $d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread "$@" > $d/pytest.log 2>&1
rc=$?; tail -5 $d/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $d/smoke.log 2>&1
rc=$?; tail -3 $d/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $d/bench.json 2> $d/bench.err
rc=$?; tail -c 600 $d/bench.json; exit $rc
