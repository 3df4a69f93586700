#!/usr/bin/env bash
# Round 6 (GPU box): instruction-cache counters of the fp32 sampler kernel
# (one one-pipe C3 step), and the counter list of this rocprofv3.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_icache
mkdir -p "$O"
timeout -k 10 120 rocprofv3 --list-avail > "$O/list_avail.txt" 2>&1 || true
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_[A-Z_]*\|SQ_INSTS_[A-Z_]*" "$O/list_avail.txt" | sort -u > "$O/names.txt" || true
timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES --kernel-include-regex fsm16_solve_kernel \
    -d "$O/pmc" -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 --f64-steps 0 \
    > "$O/bench_pmc.log" 2>&1
echo done > "$O/DONE"
