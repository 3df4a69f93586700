# round-5 fp64 held-stream check: fp64 / dropin / phases tests first, then the full suite, the default bench,
# a same-box fp64 A/B (hold8 0 / 1) and the fp64 PMC passes of the held build.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F_OUT:-r05f64}
mkdir -p "$O"
( while sleep 45; do echo "[r05f] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
echo "[r05f] fp64 tests"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "f64 or fp64 or double" tests \
    > "$O/gpu_tests_f64.log" 2>&1
echo "[r05f] full suite"
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > "$O/gpu_tests.log" 2>&1
echo "[r05f] bench"
timeout -k 10 500 python3 -u bench.py > "$O/bench.log" 2>&1
if [ -n "${F_AB:-}" ]; then
  echo "[r05f] fp64 A/B"
  cp mceik_amd/libmceik_hip.so /tmp/lib_keep.so
  for r in 1 2; do
    for v in f64hold0 f64hold1; do
      cp "mceik_amd/exp/lib_$v.so" mceik_amd/libmceik_hip.so
      timeout -k 10 300 python3 bench.py --precision 64 --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 --f64-steps 0 \
          > "$O/ab_${v}_r$r.log" 2>&1 || { cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so; exit 1; }
    done
  done
  cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so
fi
if [ -n "${F_PMC:-}" ]; then
  echo "[r05f] fp64 PMC"
  M_OUT=$(basename "$O")/m M_PRECS=64 M_TRACE=0 M_CONFIGS=0 M_REHEARSAL=0 bash tools/measure_r05.sh
fi
echo done > "$O/DONE"
