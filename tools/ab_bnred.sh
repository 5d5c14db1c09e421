for i in 1 2; do
for v in 0 1; do
  for m in f32 bf16; do
    SEG_BN_RED=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timer --math $m > gpurun_out/ab_$v_$m.log 2>&1 || exit 1
    echo "red=$v math=$m $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v_$m.log)"
  done
done
done
