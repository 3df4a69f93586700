#!/usr/bin/env bash
# Round 6, call C (GPU box): the locate3d entry-point tests, a same-box A/B of
# the SLP-vectorised build (packed v_pk_add/mul_f32, exp/lib_slp.so) against
# the default (exp/lib_cur.so) in fp32 and fp64, and the fp64 PMC record of
# the pruned fsm_kernel build (tools/measure_r05.sh passes, fp64 only).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${C_OUT:-r06_c}
mkdir -p "$O"
( while sleep 45; do echo "[r06_c] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
echo "[r06_c] locate3d tests"
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_locate3d.py \
    > "$O/gpu_tests_locate3d.log" 2>&1
echo "[r06_c] A/B fp32"
AB_VARIANTS="cur slp" AB_ROUNDS=3 AB_ARGS="--steps 3 --warmup 1 --f64-steps 0 --pipes 1" timeout -k 10 900 bash tools/ab_bench.sh
mv gpurun_out/ab "$O/ab32"
echo "[r06_c] A/B fp64"
AB_VARIANTS="cur slp" AB_ROUNDS=2 AB_ARGS="--precision 64 --steps 1 --warmup 1 --f64-steps 0 --pipes 1" \
    timeout -k 10 900 bash tools/ab_bench.sh
mv gpurun_out/ab "$O/ab64"
echo "[r06_c] fp64 PMC"
M_OUT=r06_c/m M_PRECS=64 M_TRACE=0 M_CONFIGS=0 M_REHEARSAL=0 timeout -k 10 1000 bash tools/measure_r05.sh
echo done > "$O/DONE"
