#!/usr/bin/env bash
# On the GPU box: the effective shader clock of the sampler's FSM launches
# (MI355X_MICROARCH.md "DVFS give-back": GRBM_GUI_ACTIVE / 8 / kernel wall
# time).  One GRBM pass per precision over the one-pipe C3 bench; the bench
# line of the same run gives the launch time.  Out: gpurun_out/${C_OUT:-clk}/
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${C_OUT:-clk}
mkdir -p "$O"
for prec in ${CLK_PRECS:-32 64}; do
  if [ $prec = 32 ]; then K=fsm16_solve_kernel; else K="fsm_solve_kernel<double, 2, true"; fi
  echo "[clock_probe] fp$prec $(date +%T)"
  MCEIK_LAUNCH_REPORT=1 timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$K" -d "$O/f$prec" -o pmc \
      --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 --precision $prec \
      --f64-steps 0 > "$O/bench_f$prec.log" 2>&1
  python3 - "$O" $prec "$K" <<'EOF' | tee -a "$O/summary.txt"
import csv, glob, json, os, sys
o, prec, k = sys.argv[1], sys.argv[2], sys.argv[3]
tot, disp = {}, {}
for f in glob.glob(os.path.join(o, "f" + prec, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            disp.setdefault(r["Counter_Name"], set()).add(r["Dispatch_Id"])
line = [l for l in open(os.path.join(o, "bench_f%s.log" % prec)) if l.startswith("{")][-1]
ms = json.loads(line)["roofline"]["avg_launch_ms"]
g = tot["GRBM_GUI_ACTIVE"] / len(disp["GRBM_GUI_ACTIVE"])
print(f"fp{prec}: GRBM_GUI_ACTIVE {g:.4e} per dispatch ({len(disp['GRBM_GUI_ACTIVE'])} dispatches), "
      f"launch {ms:.1f} ms -> effective clock {g / 8 / (ms * 1e-3) / 1e9:.3f} GHz")
EOF
done
