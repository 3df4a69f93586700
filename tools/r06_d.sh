#!/usr/bin/env bash
# Round 6, call D (GPU box): the fp64 sampler's throughput against its pipe
# count and timed-step count (is the line's 2-step f64 record a steady-state
# figure?), same box.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${D_OUT:-r06_d}
mkdir -p "$O"
( while sleep 45; do echo "[r06_d] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
for cfg in "2 2" "4 2" "2 3" "4 3" "2 1"; do
  set -- $cfg
  echo "[r06_d] fp64 steps $1 pipes $2"
  timeout -k 10 400 python3 bench.py --precision 64 --steps $1 --warmup 1 --pipes $2 --no-cpu-baseline --f64-steps 0 \
      > "$O/bench_f64_s$1_p$2.log" 2>&1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['frac'])" \
      "$O/bench_f64_s$1_p$2.log" $1 $2 | tee -a "$O/summary.txt"
done
echo done > "$O/DONE"
