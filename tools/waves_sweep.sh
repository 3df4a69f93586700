#!/usr/bin/env bash
# Resident waves per CU vs throughput and L2->fabric traffic (GPU box, via
# gpurun): for each W in WAVES (default "8 6 4"), one short bench run and one
# FETCH_SIZE + one WRITE_SIZE pass over the FSM kernel.  Output: gpurun_out/waves/.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/waves
mkdir -p "$OUT"
ARGS=${WS_ARGS:---steps 1 --warmup 1 --no-cpu-baseline}
for w in ${WAVES:-8 6 4}; do
  export MCEIK_WAVES_PER_CU=$w
  timeout -k 10 300 python3 bench.py $ARGS > "$OUT/w$w.log" 2>&1
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex fsm_solve_kernel -d "$OUT/w${w}_$C" -o pmc \
        --output-format csv -- python3 bench.py $ARGS > "$OUT/w${w}_$C.log" 2>&1
  done
  python3 - "$OUT" "$w" <<'PY'
import csv, glob, json, sys
out, w = sys.argv[1], sys.argv[2]
line = json.loads(open(f"{out}/w{w}.log").read().strip().splitlines()[-1])
tot = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = []
    for f in glob.glob(f"{out}/w{w}_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c:
                vals.append(float(r["Counter_Value"]))
    tot[c] = max(vals) if vals else float("nan")      # KB per dispatch (largest = the step's FSM launch)
print(f"waves/CU {w}: {line['value']:.1f} proposals/s, FSM {line['roofline']['avg_launch_ms']:.0f} ms, "
      f"FETCH x2 {2 * tot['FETCH_SIZE'] * 1024 / 1e12:.2f} TB, WRITE {tot['WRITE_SIZE'] * 1024 / 1e12:.2f} TB")
PY
done
