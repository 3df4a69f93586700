#!/usr/bin/env bash
# Round 6 (GPU box): LDS counters of the fp32 and fp64 sampler kernels (one one-pipe C3 step each).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${L_OUT:-r06_lds}
mkdir -p "$O"
C="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL"
timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex fsm16_solve_kernel -d "$O/f32" -o pmc --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 --f64-steps 0 > "$O/bench_f32.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc $C --kernel-include-regex "fsm_solve_kernel<double" -d "$O/f64" -o pmc --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 --precision 64 --f64-steps 0 > "$O/bench_f64.log" 2>&1
echo done > "$O/DONE"
