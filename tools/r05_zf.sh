# round-5 z-face copies check: the full GPU suite, then same-box A/Bs of zf0 (held streams reading the
# z-boundary nodes from the field) and zf1 (from the z-face copies), fp32 and fp64, then the default bench.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F_OUT:-r05zf}
mkdir -p "$O"
( while sleep 45; do echo "[r05zf] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
echo "[r05zf] full suite"
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > "$O/gpu_tests.log" 2>&1
echo "[r05zf] A/B fp32"
AB_VARIANTS="${F_VARIANTS:-zf0 zf1}" AB_ROUNDS=2 AB_ARGS="--steps 3 --warmup 1 --f64-steps 0 --pipes 1" \
    timeout -k 10 600 bash tools/ab_bench.sh
mv gpurun_out/ab "$O/ab32"
echo "[r05zf] A/B fp64"
AB_VARIANTS="${F_VARIANTS:-zf0 zf1}" AB_ROUNDS=2 AB_ARGS="--precision 64 --steps 1 --warmup 1 --f64-steps 0 --pipes 1" \
    timeout -k 10 600 bash tools/ab_bench.sh
mv gpurun_out/ab "$O/ab64"
echo "[r05zf] bench"
timeout -k 10 500 python3 -u bench.py > "$O/bench.log" 2>&1
echo done > "$O/DONE"
