# round-4 closing evidence on one box: smoke, the default bench line (fp32 headline + f64 record),
# rocprofv3 kernel-trace stats of the same command, the two-rank rehearsal line.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F_OUT:-r04final}
mkdir -p "$O"
( while sleep 45; do echo "[r04_final] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
echo "[r04_final] smoke"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
echo "[r04_final] bench"
timeout -k 10 500 python3 -u bench.py > "$O/bench.log" 2>&1
echo "[r04_final] trace"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/trace" -o trace --output-format csv -- \
    python3 bench.py --no-cpu-baseline > "$O/bench_under_trace.log" 2>&1
echo "[r04_final] rehearsal"
MCEIK_BENCH_REHEARSAL=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > "$O/bench_rehearsal_n2.log" 2>&1
echo done > "$O/DONE"
