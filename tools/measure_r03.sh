#!/usr/bin/env bash
# On the GPU box: the r03 evidence set for the current kernel.
#  1 rocprofv3 kernel-trace stats of the default bench (2 pipes)
#  2 PMC passes (one pipe, the timed launch): FETCH_SIZE; WRITE_SIZE; SQ VALU/LDS
#  3 a one-pipe bench line with the raw visit counters (wave steps)
#  4 relocation: bench + kernel trace + PMC (VALU/LDS) of mceik_relocate
# Outputs under gpurun_out/${M_OUT:-m03}/ (M_RELOC=0 skips 4).  Every step under its own time limit.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${M_OUT:-m03}
mkdir -p "$O"
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$O/trace" -o trace --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_under_trace.log" 2>&1
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --pipes 1 --raw-stats > "$O/bench_pipes1_raw.log" 2>&1
i=0
for P in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "fsm16_solve_kernel" -d "$O/pmc$i" -o pmc \
      --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 > "$O/bench_pmc$i.log" 2>&1
done
if [ "${M_RELOC:-1}" = 1 ]; then
timeout -k 10 200 python3 tools/bench_relocate.py > "$O/relocate.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/reloc_trace" -o trace --output-format csv -- \
    python3 tools/bench_relocate.py --iters 5 > "$O/relocate_under_trace.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    --kernel-include-regex "relocate_lds_kernel" -d "$O/reloc_pmc" -o pmc --output-format csv -- \
    python3 tools/bench_relocate.py --iters 2 > "$O/relocate_pmc.log" 2>&1
fi
timeout -k 10 420 python3 bench.py > "$O/bench_default.log" 2>&1
echo done > "$O/DONE"
