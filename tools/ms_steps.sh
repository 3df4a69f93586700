set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mss
for n in 3 10 24; do for m in 0 1; do
  MCEIK_PERSIST=$m timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $n > gpurun_out/mss/p${m}_s$n.log 2>&1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('persist', sys.argv[2], 'steps', sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/mss/p${m}_s$n.log $m $n | tee -a gpurun_out/mss/summary.txt
done; done
