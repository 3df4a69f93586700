# requested bytes by category (the -DMCEIK_TRAFFIC accounting build, mceik_amd/exp/lib_traffic.so) of the
# fp32 and fp64 one-pipe launches
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F_OUT:-r05trf}
mkdir -p "$O"
cp mceik_amd/libmceik_hip.so /tmp/lib_keep.so
cp mceik_amd/exp/lib_traffic.so mceik_amd/libmceik_hip.so
for prec in 32 64; do
  timeout -k 10 300 python3 bench.py --precision $prec --steps 1 --warmup 0 --no-cpu-baseline --pipes 1 --f64-steps 0 \
      --raw-stats > "$O/bench_f${prec}_traffic_build.log" 2>&1 || { cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so; exit 1; }
done
cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so
echo done > "$O/DONE"
