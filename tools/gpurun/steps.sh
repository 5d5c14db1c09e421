#!/bin/bash
# Run GPU steps in order, each under its own time limit; a plain test failure (rc 1) is
# reported and the next step runs, anything worse (fault, abort, timeout) ends the call.
#   steps.sh <tag> "<name>|<seconds>|<command>" ...
tag=$1; shift
d=gpurun_out/$tag; mkdir -p $d
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 $secs bash -c "$cmd" > $d/$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -n 4 $d/$name.log
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
