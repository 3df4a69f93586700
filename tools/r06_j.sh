#!/usr/bin/env bash
# Round 6, call J (GPU box): same-box fp64 A/B of the z-major rows (exp/lib_lds.so) against
# v41 (exp/lib_base.so): one pipe and the f64 record's two pipes.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_j
mkdir -p "$O"
( while sleep 45; do echo "[r06_j] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
AB_VARIANTS="base lds" AB_ROUNDS=2 AB_ARGS="--precision 64 --steps 1 --warmup 1 --f64-steps 0 --pipes 1" timeout -k 10 600 bash tools/ab_bench.sh
mv gpurun_out/ab "$O/ab64_pipes1"
AB_VARIANTS="base lds" AB_ROUNDS=2 AB_ARGS="--precision 64 --steps 2 --warmup 1 --f64-steps 0" timeout -k 10 700 bash tools/ab_bench.sh
mv gpurun_out/ab "$O/ab64_pipes2"
echo done > "$O/DONE"
