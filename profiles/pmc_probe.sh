#!/usr/bin/env bash
# Runs on the GPU box (via gpurun): several single-group PMC passes over the
# bench (FSM kernel only) to attribute time and traffic.  Output:
# gpurun_out/probe_<tag>/pass<i>/.  usage: profiles/pmc_probe.sh <tag> [bench args]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/probe_$TAG
mkdir -p "$OUT"
PASSES=(
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INSTS_VALU"
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
  "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES"
)
# PASS_SEL="1 3" limits the run to those passes
SEL=${PASS_SEL:-}
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  if [ -n "$SEL" ] && [[ " $SEL " != *" $i "* ]]; then continue; fi
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "${KREGEX:-fsm16_solve_kernel}" -d "$OUT/pass$i" -o pmc --output-format csv -- \
      python3 bench.py "$@" > "$OUT/bench_pass$i.log" 2>&1
done
find "$OUT" -name '*counter_collection.csv'
