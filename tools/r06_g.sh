#!/usr/bin/env bash
# Round 6, call G (GPU box): the round-trip-lean held-stream decision (exp/lib_hd2.so):
# its parity tests, a same-box fp32 A/B against the v40 build (exp/lib_base.so),
# and the phase clocks of the instrumented build (exp/lib_pclk.so).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${G_OUT:-r06_g}
mkdir -p "$O"
( while sleep 45; do echo "[r06_g] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
F_OUT=${G_OUT:-r06_g} F_CAND=${G_CAND:-hd2} F_TESTS="tests/test_gpu_hold.py tests/test_gpu_fsm.py tests/test_gpu_mcmc.py tests/test_gpu_configs.py" \
    F_V32="${G_V32:-base hd2}" F_V64="${G_V64:-}" F_ROUNDS=${G_ROUNDS:-3} timeout -k 10 1000 bash tools/r05_ab.sh
P_OUT=${G_OUT:-r06_g}/pclk timeout -k 10 400 bash tools/r06_pclk.sh
echo done > "$O/DONE"
