# round-5 same-box A/B of library variants (mceik_amd/exp/lib_<v>.so): fp32 and fp64 one-pipe launches,
# after the parity tests of the candidate variant (F_CAND, run in place).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F_OUT:-r05ab}
mkdir -p "$O"
( while sleep 45; do echo "[r05ab] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
cp mceik_amd/libmceik_hip.so /tmp/lib_keep.so
if [ -n "${F_CAND:-}" ]; then
  echo "[r05ab] parity tests of $F_CAND"
  cp "mceik_amd/exp/lib_$F_CAND.so" mceik_amd/libmceik_hip.so
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
      ${F_TESTS:-tests/test_gpu_fsm.py tests/test_gpu_configs.py tests/test_gpu_mcmc.py} > "$O/gpu_tests_$F_CAND.log" 2>&1 \
      || { cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so; exit 1; }
  cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so
fi
if [ -n "${F_V32:-}" ]; then
  echo "[r05ab] A/B fp32"
  AB_VARIANTS="$F_V32" AB_ROUNDS=${F_ROUNDS:-2} AB_ARGS="--steps 3 --warmup 1 --f64-steps 0 --pipes 1" timeout -k 10 900 bash tools/ab_bench.sh
  mv gpurun_out/ab "$O/ab32"
fi
if [ -n "${F_V64:-}" ]; then
  echo "[r05ab] A/B fp64"
  AB_VARIANTS="$F_V64" AB_ROUNDS=${F_ROUNDS:-2} AB_ARGS="--precision 64 --steps 1 --warmup 1 --f64-steps 0 --pipes 1" \
      timeout -k 10 900 bash tools/ab_bench.sh
  mv gpurun_out/ab "$O/ab64"
fi
cp /tmp/lib_keep.so mceik_amd/libmceik_hip.so
echo done > "$O/DONE"
