#!/usr/bin/env bash
# A/B on the GPU box: "<variant>:<MCEIK_PERSIST>:<pipes>" entries of MS_AB,
# interleaved rounds, one short bench line each.  Outputs under gpurun_out/msab/.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/msab
mkdir -p "$O"
cp mceik_amd/libmceik_hip.so /tmp/keep.so
for r in $(seq 1 "${MS_ROUNDS:-2}"); do
  for e in $MS_AB; do
    IFS=: read -r v m p <<< "$e"
    cp "mceik_amd/exp/lib_$v.so" mceik_amd/libmceik_hip.so
    MCEIK_PERSIST=$m timeout -k 10 300 python3 bench.py --steps ${MS_STEPS:-3} --warmup 1 --no-cpu-baseline --pipes $p > "$O/${v}_${m}_${p}_r$r.log" 2>&1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$O/${v}_${m}_${p}_r$r.log" "$e" | tee -a "$O/summary.txt"
  done
done
cp /tmp/keep.so mceik_amd/libmceik_hip.so
