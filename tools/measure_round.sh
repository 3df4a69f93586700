#!/usr/bin/env bash
# Runs on the GPU box (gpurun) from the repo root: the evidence set for one
# kernel revision, outputs under gpurun_out/meas_<tag>/ (copy what is judged
# into profiles/<tag>/).  Steps stop at the first failure.
#   1 full GPU test suite            2 rocprofv3 stats + FETCH/WRITE passes (profiles/collect.sh)
#   3 accounting build (requested bytes by category; mceik_amd/exp/lib_traffic.so)
#   4 C2, C5 and fp64 C3 bench lines  5 the default bench (with the CPU baseline)
# usage: tools/measure_round.sh <tag>
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1
O=gpurun_out/meas_$TAG
mkdir -p "$O"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
bash profiles/collect.sh "$TAG" --steps 2 --warmup 1 --no-cpu-baseline > "$O/collect.log" 2>&1
if [ -f mceik_amd/exp/lib_traffic.so ]; then
  cp mceik_amd/libmceik_hip.so /tmp/lib_keep.so
  cp mceik_amd/exp/lib_traffic.so mceik_amd/libmceik_hip.so
  timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$O/bench_traffic_build.log" 2>&1 || { cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so; exit 1; }
  cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so
fi
timeout -k 10 200 python3 bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_c2.log" 2>&1
timeout -k 10 300 python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline > "$O/bench_c5.log" 2>&1
timeout -k 10 300 python3 bench.py --precision 64 --steps 1 --warmup 1 --no-cpu-baseline > "$O/bench_c3_fp64.log" 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 400 python3 bench.py > "$O/bench_default.log" 2>&1
echo done > "$O/DONE"
