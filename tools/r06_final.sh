#!/usr/bin/env bash
# Round 6 closing evidence at HEAD (GPU box): the full GPU suite and smoke,
# the default bench line with the driver's arguments, the same command's
# rocprofv3 kernel-trace stats (the FSM kernels' average launch times), C2 / C5
# lines, and the 8-rank rehearsal through bench.py's own launcher.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${E_OUT:-r06_final}
mkdir -p "$O"
( while sleep 45; do echo "[r06_final] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
if [ "${E_TESTS:-1}" = 1 ]; then
echo "[r06_final] gpu tests"
timeout -k 10 1100 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
    > "$O/gpu_tests.log" 2>&1
echo "[r06_final] smoke"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
fi
echo "[r06_final] bench (driver arguments)"
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.log" 2>&1
echo "[r06_final] bench under the kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace" -o trace --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --f64-steps 2 > "$O/bench_under_trace.log" 2>&1
if [ "${E_CONFIGS:-1}" = 1 ]; then
echo "[r06_final] C2 / C5"
timeout -k 10 300 python3 bench.py --config C2 --steps 10 --warmup 1 --no-cpu-baseline --f64-steps 0 > "$O/bench_c2.log" 2>&1
timeout -k 10 400 python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --pipes 1 --f64-steps 0 \
    > "$O/bench_c5.log" 2>&1
echo "[r06_final] 8-rank rehearsal"
MCEIK_BENCH_REHEARSAL=1 timeout -k 10 600 python3 bench.py --gpus 8 --chains 32 --steps 2 --warmup 1 \
    > "$O/bench_rehearsal_n8.log" 2>&1
fi
echo done > "$O/DONE"
