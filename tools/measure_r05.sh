#!/usr/bin/env bash
# On the GPU box: the r05 evidence set for the current kernels.
#  1 rocprofv3 kernel-trace stats of the default bench (fp32 two pipes + the fp64 record)
#  2 fp32, one pipe, the timed launch: raw visit counters, PMC FETCH_SIZE; WRITE_SIZE; SQ; SQ issue + clock
#  3 fp64 (--precision 64), one pipe: the same
#  4 the N = 2 flow rehearsed on one GPU (MCEIK_BENCH_REHEARSAL=1, gloo)
# Outputs under gpurun_out/${M_OUT:-m05}/.  Every step under its own time limit.
# M_PRECS (default "32 64"), M_TRACE / M_REHEARSAL (default 1) select the parts.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${M_OUT:-m05}
mkdir -p "$O"
( while sleep 45; do echo "[measure_r05] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES"
# issue breakdown (quad-cycles summed over waves) + the effective clock (GRBM_GUI_ACTIVE / 8 / launch time)
SQ2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
if [ "${M_TRACE:-1}" = 1 ]; then
echo "[measure_r05] trace"
timeout -k 10 480 rocprofv3 --kernel-trace --stats -d "$O/trace" -o trace --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --f64-steps 2 > "$O/bench_under_trace.log" 2>&1
fi
for prec in ${M_PRECS:-32 64}; do
  if [ $prec = 32 ]; then K=fsm16_solve_kernel; else K="fsm_solve_kernel<double, 2, true"; fi
  echo "[measure_r05] fp$prec raw"
  timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 --raw-stats --precision $prec \
      > "$O/bench_f${prec}_pipes1_raw.log" 2>&1
  i=0
  for P in FETCH_SIZE WRITE_SIZE "$SQ" "$SQ2"; do
    i=$((i+1))
    echo "[measure_r05] fp$prec pmc$i"
    timeout -k 10 400 rocprofv3 --pmc $P --kernel-include-regex "$K" -d "$O/f${prec}_pmc$i" -o pmc \
        --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 --precision $prec \
        > "$O/bench_f${prec}_pmc$i.log" 2>&1
  done
done
if [ "${M_CONFIGS:-1}" = 1 ]; then
  echo "[measure_r05] C2 / C5"
  timeout -k 10 300 python3 bench.py --config C2 --steps 10 --warmup 1 --no-cpu-baseline --f64-steps 0 > "$O/bench_c2.log" 2>&1
  timeout -k 10 400 python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --pipes 1 --f64-steps 0 \
      > "$O/bench_c5.log" 2>&1
fi
[ "${M_REHEARSAL:-1}" = 1 ] || { echo done > "$O/DONE"; exit 0; }
echo "[measure_r05] rehearsal (bench.py's own --gpus launcher)"
MCEIK_BENCH_REHEARSAL=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 2 --warmup 1 > "$O/bench_rehearsal_n2.log" 2>&1
echo done > "$O/DONE"
