#!/usr/bin/env bash
# Round 6, call A (on the GPU box): C4 readiness rehearsal with 8 ranks through
# bench.py's own --gpus launcher (one GPU shared, gloo), the fp32-vs-fp64
# accept agreement at C3 + the tolerance tests, and a short default bench.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${A_OUT:-r06_a}
mkdir -p "$O"
( while sleep 45; do echo "[r06_a] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
if [ "${A_REH:-1}" = 1 ]; then
echo "[r06_a] 8-rank rehearsal"
MCEIK_BENCH_REHEARSAL=1 timeout -k 10 600 python3 bench.py --gpus 8 --chains 32 --steps 2 --warmup 1 \
    > "$O/bench_rehearsal_n8.log" 2>&1
fi
if [ "${A_TOL:-1}" = 1 ]; then
echo "[r06_a] tolerance / accept tests"
timeout -k 10 1000 python3 -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu \
    ${A_TESTS:-tests/test_gpu_tolerance.py} > "$O/gpu_tests_tolerance.log" 2>&1
fi
if [ "${A_BENCH:-1}" = 1 ]; then
echo "[r06_a] bench"
timeout -k 10 400 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --f64-steps 1 > "$O/bench.log" 2>&1
fi
echo done > "$O/DONE"
