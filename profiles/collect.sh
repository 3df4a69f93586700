#!/usr/bin/env bash
# Runs on the GPU box (via gpurun) from the repo root: kernel-trace stats of the
# bench command, then one PMC pass per HBM counter (FETCH_SIZE and WRITE_SIZE
# do not fit in one pass on gfx950).  Outputs go to gpurun_out/prof_<tag>/.
# usage: profiles/collect.sh <tag> [bench args...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
ARGS=("$@")
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- \
    python3 bench.py "${ARGS[@]}" > "$OUT/bench_under_trace.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 900 rocprofv3 --pmc $C -d "$OUT/pmc_$C" -o pmc --output-format csv -- \
      python3 bench.py "${ARGS[@]}" > "$OUT/bench_pmc_$C.log" 2>&1
done
find "$OUT" -name '*.csv' | head -50
