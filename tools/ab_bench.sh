#!/usr/bin/env bash
# A/B throughput of prebuilt library variants on the GPU box (interleaved
# rounds, same box): for each round and variant mceik_amd/exp/lib_<v>.so, one
# short default bench run (no CPU baseline); prints "<variant> <proposals/s>".
# usage: AB_VARIANTS="a b" AB_ROUNDS=2 AB_ARGS="--steps 2 --warmup 1" tools/ab_bench.sh
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab
mkdir -p "$OUT"
cp mceik_amd/libmceik_hip.so /tmp/lib_keep.so
for r in $(seq 1 "${AB_ROUNDS:-2}"); do
  for v in ${AB_VARIANTS}; do
    cp "mceik_amd/exp/lib_$v.so" mceik_amd/libmceik_hip.so
    timeout -k 10 300 python3 bench.py ${AB_ARGS:---steps 2 --warmup 1} --no-cpu-baseline > "$OUT/${v}_r$r.log" 2>&1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_launch_ms'])" "$OUT/${v}_r$r.log" "$v" | tee -a "$OUT/summary.txt"
  done
done
cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so
