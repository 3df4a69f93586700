#!/usr/bin/env bash
# Round 6, call F (GPU box): the wave-priority phases (v40 / v37c).
#  part 1: the full GPU suite, smoke and the default bench line
#  part 2: the PMC record of both kernels (tools/measure_r05.sh: kernel trace,
#          FETCH / WRITE / SQ passes per precision, C2 / C5)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F_OUT:-r06_f}
mkdir -p "$O"
( while sleep 45; do echo "[r06_f] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
if [ "${F_PART:-1}" = 1 ]; then
  echo "[r06_f] gpu tests"
  timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
      > "$O/gpu_tests.log" 2>&1
  echo "[r06_f] smoke"
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  echo "[r06_f] bench (driver arguments)"
  timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.log" 2>&1
else
  M_OUT=${F_OUT:-r06_f}/m M_PRECS="${F_PRECS:-32 64}" M_TRACE=1 M_CONFIGS=1 M_REHEARSAL=0 timeout -k 10 1100 bash tools/measure_r05.sh
fi
echo done > "$O/DONE"
