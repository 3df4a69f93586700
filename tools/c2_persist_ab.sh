set -euo pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c2ab
for r in 1 2; do for m in 0 1; do
  MCEIK_PERSIST=$m timeout -k 10 200 python3 bench.py --config C2 --no-cpu-baseline > gpurun_out/c2ab/c2_p${m}_r$r.log 2>&1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C2 persist'+sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/c2ab/c2_p${m}_r$r.log $m | tee -a gpurun_out/c2ab/summary.txt
done; done
