# round-5 closing evidence at the head: smoke, the full GPU suite, the default bench line, the rocprofv3
# kernel-trace stats of the same command, the fp32/fp64 PMC passes (tools/measure_r05.sh) and the C2/C5
# lines.  F_PARTS selects: s(moke) t(ests) b(ench) r(trace) p(mc) c(onfigs).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F_OUT:-r05close}
P=${F_PARTS:-stbr}
mkdir -p "$O"
( while sleep 45; do echo "[r05c] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
if [[ $P == *s* ]]; then echo "[r05c] smoke"; timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; fi
if [[ $P == *t* ]]; then echo "[r05c] tests"; timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > "$O/gpu_tests.log" 2>&1; fi
if [[ $P == *b* ]]; then echo "[r05c] bench"; timeout -k 10 500 python3 -u bench.py > "$O/bench.log" 2>&1; fi
if [[ $P == *r* ]]; then
  echo "[r05c] trace"
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/trace" -o trace --output-format csv -- \
      python3 bench.py --no-cpu-baseline > "$O/bench_under_trace.log" 2>&1
fi
if [[ $P == *p* ]]; then echo "[r05c] pmc"; M_OUT=$(basename "$O")/m M_TRACE=0 M_CONFIGS=0 M_REHEARSAL=0 bash tools/measure_r05.sh; fi
if [[ $P == *c* ]]; then
  echo "[r05c] C2 / C5"
  timeout -k 10 300 python3 bench.py --config C2 --steps 10 --warmup 1 --no-cpu-baseline --f64-steps 0 > "$O/bench_c2.log" 2>&1
  timeout -k 10 400 python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --pipes 1 --f64-steps 0 \
      > "$O/bench_c5.log" 2>&1
fi
echo done > "$O/DONE"
