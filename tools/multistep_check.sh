#!/usr/bin/env bash
# On the GPU box: multi-step launch tests, the full GPU suite, then an A/B of
# multi-step vs per-step (two pipes) bench lines.  Outputs under gpurun_out/ms/.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${MS_OUT:-ms}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_multistep.py -x -v --timeout 200 --timeout-method thread > "$O/tests_multistep.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 850 --timeout-method thread > "$O/gpu_tests.log" 2>&1
for r in 1 2; do
  for m in 0 1; do
    MCEIK_PERSIST=$m timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_persist${m}_r$r.log" 2>&1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('persist'+sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'])" "$O/bench_persist${m}_r$r.log" $m | tee -a "$O/summary.txt"
  done
done
