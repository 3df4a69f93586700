set -e
mkdir -p gpurun_out/ab
for w in 8 7 6 4; do
  MCEIK_WAVES_PER_CU=$w timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/w$w.log 2>&1
done
