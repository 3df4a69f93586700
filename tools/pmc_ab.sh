#!/usr/bin/env bash
# A/B PMC probe on the GPU box: for each prebuilt variant mceik_amd/exp/lib_<v>.so,
# one rocprofv3 --pmc pass per counter group over a short bench run (FSM kernel
# only).  usage: AB_VARIANTS="a b" PMC_GROUPS="C1 C2;C3 C4" tools/pmc_ab.sh
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_ab
mkdir -p "$OUT"
cp mceik_amd/libmceik_hip.so /tmp/lib_keep.so
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS}"
for v in ${AB_VARIANTS}; do
  cp mceik_amd/exp/lib_$v.so mceik_amd/libmceik_hip.so
  mkdir -p "$OUT/$v"
  i=0
  for P in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "fsm16_solve_kernel|fsm_solve_kernel" -d "$OUT/$v/pass$i" -o pmc \
        --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 > "$OUT/$v/bench_pass$i.log" 2>&1
  done
done
cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so
