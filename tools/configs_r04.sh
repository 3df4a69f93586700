#!/usr/bin/env bash
# On the GPU box: the other BASELINE configurations with the round-4 build --
# C2 (64^3, 256 chains x 16 stations) and C5 (256^3, 256 chains x 64 stations,
# one pipe).  gpurun_out/${C_OUT:-cfg04}/.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${C_OUT:-cfg04}
mkdir -p "$O"
timeout -k 10 300 python3 bench.py --config C2 --steps 10 --warmup 1 --no-cpu-baseline --f64-steps 0 > "$O/bench_c2.log" 2>&1
timeout -k 10 400 python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --pipes 1 --f64-steps 0 \
    > "$O/bench_c5_pipes1.log" 2>&1
echo done > "$O/DONE"
