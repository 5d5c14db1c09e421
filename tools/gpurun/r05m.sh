#!/bin/bash
# Round-5 evidence at HEAD: roofline profiles (kernel trace + FETCH / WRITE / MFMA PMC passes) of both maths with the
# contention tables, the UNet configs[4] bf16io profile, and the default bench line.
t=${1:-r05m}
d=gpurun_out/$t; mkdir -p $d
export TMPDIR=/tmp SEG_COMMIT=$(cat .commit 2>/dev/null)
for m in f32 bf16io; do
  bash tools/gpurun/roof.sh ${t}_$m --math $m || exit 1
  python tools/queues.py gpurun_out/${t}_$m/prof/run_kernel_trace.csv > gpurun_out/${t}_$m/queues.txt || exit 1
  SEG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${t}_$m/alone -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-timer --no-bf16io-block --no-infer-block --no-unet-block --math $m > gpurun_out/${t}_$m/alone.log 2>&1 || exit 1
  python tools/contention.py gpurun_out/${t}_$m/prof/run_kernel_trace.csv gpurun_out/${t}_$m/alone/run_kernel_trace.csv --md gpurun_out/${t}_$m/contention.md > /dev/null || exit 1
  echo "== $m profiled"
done
ROOF_MODEL=UNet bash tools/gpurun/roof.sh ${t}_unet --math bf16io --model UNet --height 512 --width 1024 --batch 8 || exit 1
python tools/queues.py gpurun_out/${t}_unet/prof/run_kernel_trace.csv > gpurun_out/${t}_unet/queues.txt || exit 1
timeout -k 10 400 python bench.py > $d/bench.json 2> $d/bench.err || { tail -5 $d/bench.err; exit 1; }
tail -c 400 $d/bench.json
