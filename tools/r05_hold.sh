# round-5 held-stream check: fsm16 parity first (stop at the first failure), the full GPU suite,
# the default bench line, then a same-box A/B of the old (hold0) and held (hold1) streams.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F_OUT:-r05hold}
mkdir -p "$O"
( while sleep 45; do echo "[r05h] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
echo "[r05h] fsm tests"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fsm.py \
    > "$O/gpu_tests_fsm.log" 2>&1
echo "[r05h] full suite"
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
    > "$O/gpu_tests.log" 2>&1
echo "[r05h] bench"
timeout -k 10 500 python3 -u bench.py > "$O/bench.log" 2>&1
if [ -n "${F_AB:-}" ]; then
  echo "[r05h] A/B"
  AB_VARIANTS="hold0 hold1" AB_ROUNDS=2 AB_ARGS="--steps 3 --warmup 1 --f64-steps 0" timeout -k 10 900 bash tools/ab_bench.sh
  cp -r gpurun_out/ab "$O/ab"
fi
echo done > "$O/DONE"
