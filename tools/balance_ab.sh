#!/usr/bin/env bash
# Same-box A/B of the C3 step modes at the default 10 timed steps: two pipes
# (per-step launches), multi-step launches with cost-balanced chain groups,
# multi-step launches with 8 contiguous groups.  Prints "<mode> <proposals/s> <ms/step>".
# usage (GPU box): tools/balance_ab.sh [rounds] [bench args...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bal
mkdir -p "$O"
R=${1:-2}; shift || true
for r in $(seq 1 "$R"); do
  for m in pipes2 ms_bal ms_flat; do
    case $m in
      pipes2) env_="MCEIK_PERSIST=0" ;;
      ms_bal) env_="MCEIK_PERSIST=1" ;;
      ms_flat) env_="MCEIK_PERSIST=1 MCEIK_MC_BALANCE=0" ;;
    esac
    env $env_ timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$O/${m}_r$r.log" 2>&1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$O/${m}_r$r.log" "$m" | tee -a "$O/summary.txt"
  done
done
