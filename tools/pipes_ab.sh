#!/usr/bin/env bash
# On the GPU box: interleaved bench runs of the default library with 1, 2 and
# 3 pipes (PIPES_LIST), AB_ROUNDS rounds; prints "<pipes> <proposals/s> <ms/step>".
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pipes_ab
mkdir -p "$OUT"
for r in $(seq 1 "${AB_ROUNDS:-2}"); do
  for p in ${PIPES_LIST:-1 2 3}; do
    timeout -k 10 300 python3 bench.py --steps ${AB_STEPS:-3} --warmup 1 --no-cpu-baseline --pipes $p ${AB_EXTRA:-} > "$OUT/p${p}_r$r.log" 2>&1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/p${p}_r$r.log" "$p" | tee -a "$OUT/summary.txt"
  done
done
