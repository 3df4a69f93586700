#!/usr/bin/env bash
# Round 6, call H (GPU box): the fp64 neighbour rows in z-major layout (exp/lib_lds.so):
# the full GPU suite on it, a same-box fp64 A/B against HEAD (exp/lib_base.so), and its
# LDS counters (tools/r06_lds.sh passes, fp64).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${H_OUT:-r06_h}
mkdir -p "$O"
( while sleep 45; do echo "[r06_h] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
F_OUT=${H_OUT:-r06_h} F_CAND=${H_CAND:-lds} F_TESTS="tests" F_V64="base ${H_CAND:-lds}" F_ROUNDS=2 \
    timeout -k 10 1100 bash tools/r05_ab.sh
cp mceik_amd/libmceik_hip.so /tmp/lib_keep2.so
cp mceik_amd/exp/lib_${H_CAND:-lds}.so mceik_amd/libmceik_hip.so
C="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL"
rc=0
timeout -s KILL 400 rocprofv3 --pmc $C --kernel-include-regex "fsm_solve_kernel<double" -d "$O/lds64" -o pmc --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 --precision 64 --f64-steps 0 > "$O/bench_lds64.log" 2>&1 || rc=$?
cp /tmp/lib_keep2.so mceik_amd/libmceik_hip.so
[ $rc = 0 ] || exit $rc
echo done > "$O/DONE"
