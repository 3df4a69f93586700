set -e
mkdir -p gpurun_out/ab
cp mceik_amd/libmceik_hip.so /tmp/lib_keep.so
for v in ${AB_VARIANTS:-base q2b lq2b}; do
  cp mceik_amd/exp/lib_$v.so mceik_amd/libmceik_hip.so
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/b_$v.log 2>&1
done
cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so
