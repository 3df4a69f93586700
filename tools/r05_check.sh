# round-5 check on one box: the changed GPU tests, the --gpus 2 rehearsal through
# bench.py's own launcher, and the default bench line.  F_OUT names the output dir;
# F_TESTS the pytest selection (default: the tests this round touched).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F_OUT:-r05a}
mkdir -p "$O"
( while sleep 45; do echo "[r05] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
echo "[r05] tests"
timeout -k 10 1500 python3 -u -m pytest -x -v -s --timeout 1200 --timeout-method thread -m gpu \
    ${F_TESTS:-tests/test_gpu_tolerance.py tests/test_gpu_phases.py tests/test_gpu_multistep.py} > "$O/gpu_tests.log" 2>&1
echo "[r05] rehearsal --gpus 2"
MCEIK_BENCH_REHEARSAL=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 2 --warmup 1 > "$O/bench_rehearsal_n2.log" 2>&1
echo "[r05] bench"
timeout -k 10 500 python3 -u bench.py ${F_BENCH:-} > "$O/bench.log" 2>&1

if [ -n "${F_ADMIT:-}" ]; then
  # admission statistics (experiment build mceik_amd/exp/lib_admit.so, one-pipe launch)
  echo "[r05] admission stats"
  cp mceik_amd/libmceik_hip.so /tmp/lib_keep.so
  cp mceik_amd/exp/lib_admit.so mceik_amd/libmceik_hip.so
  timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 --raw-stats --f64-steps 0 \
      > "$O/bench_admit.log" 2>&1 || { cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so; exit 1; }
  cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so
fi
echo done > "$O/DONE2"
