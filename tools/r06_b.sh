#!/usr/bin/env bash
# Round 6, call B (GPU box): the full GPU suite + smoke on the pruned build,
# then a same-box fp64 A/B of the pre-prune library (exp/lib_prev.so) against
# the pruned one (exp/lib_cur.so): only fsm_kernel's register allocation
# differs (removed variants).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${B_OUT:-r06_b}
mkdir -p "$O"
( while sleep 45; do echo "[r06_b] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
if [ "${B_TESTS:-1}" = 1 ]; then
echo "[r06_b] gpu tests"
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu ${B_SEL:-tests} \
    > "$O/gpu_tests.log" 2>&1
echo "[r06_b] smoke"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
fi
if [ -n "${B_V64:-}" ]; then
echo "[r06_b] A/B fp64"
AB_VARIANTS="$B_V64" AB_ROUNDS=${B_ROUNDS:-2} AB_ARGS="--precision 64 --steps 1 --warmup 1 --f64-steps 0 --pipes 1" \
    timeout -k 10 900 bash tools/ab_bench.sh
mv gpurun_out/ab "$O/ab64"
fi
if [ -n "${B_V32:-}" ]; then
echo "[r06_b] A/B fp32"
AB_VARIANTS="$B_V32" AB_ROUNDS=${B_ROUNDS:-2} AB_ARGS="--steps 3 --warmup 1 --f64-steps 0 --pipes 1" \
    timeout -k 10 900 bash tools/ab_bench.sh
mv gpurun_out/ab "$O/ab32"
fi
echo done > "$O/DONE"
