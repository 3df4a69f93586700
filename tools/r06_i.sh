#!/usr/bin/env bash
# Round 6, call I (GPU box): the default bench line (driver arguments) and the fp64
# PMC record (tools/measure_r05.sh, fp64 passes) at the head.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${I_OUT:-r06_i}
mkdir -p "$O"
( while sleep 45; do echo "[r06_i] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.log" 2>&1
M_OUT=${I_OUT:-r06_i}/m M_PRECS="${I_PRECS:-64}" M_TRACE=1 M_CONFIGS=0 M_REHEARSAL=0 timeout -k 10 900 bash tools/measure_r05.sh
echo done > "$O/DONE"
