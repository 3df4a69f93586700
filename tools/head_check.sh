#!/usr/bin/env bash
# HEAD check on the GPU box: full GPU test suite, smoke, default bench.
# Outputs under gpurun_out/head/.  Steps stop at the first failure.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/head
mkdir -p "$O"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 400 python3 bench.py > "$O/bench_default.log" 2>&1
echo done > "$O/DONE"
