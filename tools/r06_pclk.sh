#!/usr/bin/env bash
# Round 6 (GPU box): phase clocks of the fp32 step (exp/lib_pclk.so, built with
# -DMCEIK_TRAFFIC -DMCEIK_PHASECLK): one one-pipe C3 step; the per-launch sums
# print on the "mceik traffic" line (categories 0..5 = step phases, fsm16_kernel.hip).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${P_OUT:-r06_pclk}
mkdir -p "$O"
cp mceik_amd/libmceik_hip.so /tmp/lib_keep.so
cp mceik_amd/exp/lib_pclk.so mceik_amd/libmceik_hip.so
rc=0
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --pipes 1 --no-cpu-baseline --f64-steps 0 > "$O/bench_pclk.log" 2>&1 || rc=$?
cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --pipes 1 --no-cpu-baseline --f64-steps 0 > "$O/bench_ref.log" 2>&1
echo done > "$O/DONE"
