#!/usr/bin/env bash
# Round 6, call K (GPU box): the fp32 kernel's held-stream decision in the fp64 kernel
# (exp/lib_hd64.so) against the head (exp/lib_base.so): fp64 two pipes, same box.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_k
mkdir -p "$O"
( while sleep 45; do echo "[r06_k] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
AB_VARIANTS="base hd64" AB_ROUNDS=2 AB_ARGS="--precision 64 --steps 2 --warmup 1 --f64-steps 0" timeout -k 10 700 bash tools/ab_bench.sh
mv gpurun_out/ab "$O/ab64_pipes2"
echo done > "$O/DONE"
