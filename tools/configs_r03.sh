#!/usr/bin/env bash
# On the GPU box: C5 with two pipes (one shared, budget-split workspace) and
# one pipe, C2, the N=2 flow rehearsed on one GPU, smoke.  gpurun_out/cfg03/.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cfg03
mkdir -p "$O"
timeout -k 10 400 python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline > "$O/bench_c5_pipes2.log" 2>&1
timeout -k 10 400 python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --pipes 1 > "$O/bench_c5_pipes1.log" 2>&1
timeout -k 10 300 python3 bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_c2.log" 2>&1
MCEIK_BENCH_REHEARSAL=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
    > "$O/bench_rehearsal_n2.log" 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
echo done > "$O/DONE"
