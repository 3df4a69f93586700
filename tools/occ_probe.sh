#!/usr/bin/env bash
# On the GPU box: sensitivity of the sampler's FSM launch to resident waves per
# CU (MCEIK_WAVES_PER_CU caps the occupancy the library computes), C3 one pipe.
# OCC_RUNS: "prec:waves ..." (waves 0 = the library's occupancy).  Out: gpurun_out/${O_OUT:-occ}/
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${O_OUT:-occ}
mkdir -p "$O"
for run in ${OCC_RUNS:-64:0 64:5 64:4 32:0 32:7 32:6}; do
  prec=${run%%:*}; w=${run#*:}
  env_cap=""; [ "$w" != 0 ] && env_cap="MCEIK_WAVES_PER_CU=$w"
  env $env_cap MCEIK_LAUNCH_REPORT=1 timeout -k 10 300 python3 bench.py --precision $prec --steps 1 --warmup 1 \
      --no-cpu-baseline --pipes 1 --f64-steps 0 > "$O/f${prec}_w$w.log" 2>&1
  python3 - "$O/f${prec}_w$w.log" "fp$prec waves/CU cap $w" <<'PY' | tee -a "$O/summary.txt"
import json, sys
txt = open(sys.argv[1]).read().splitlines()
d = json.loads([l for l in txt if l.startswith("{")][-1])
rep = sorted(set(l for l in txt if l.startswith("mceik fsm launch")))
print(sys.argv[2], d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], "|", rep[-1] if rep else "")
PY
done
