set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04_trf
cp mceik_amd/exp/lib_traffic.so mceik_amd/libmceik_hip.so
timeout -k 10 300 python3 bench.py --precision 64 --steps 1 --warmup 0 --no-cpu-baseline --pipes 1 --f64-steps 0 > gpurun_out/r04_trf/bench_f64_traffic_build.log 2>&1
