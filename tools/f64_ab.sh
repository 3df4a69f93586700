# Sampler-kernel A/B on one box: each variant's libmceik_hip.so (mceik_amd/exp/lib_<v>.so;
# v:N caps the resident waves at N) runs the C3 one-pipe bench for each precision in
# AB_PRECS (default 64) with AB_STEPS timed steps (default 1), two interleaved rounds;
# then the fp64 parity tests on each variant in F64_TEST.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F64_OUT:-f64e}
mkdir -p $O
cp mceik_amd/libmceik_hip.so /tmp/keep.so
for r in 1 2; do for vv in ${F64_VARIANTS:-f64a f64b f64c}; do
  v=${vv%%:*}; mw=0; [ "$v" != "$vv" ] && mw=${vv#*:}
  cp mceik_amd/exp/lib_$v.so mceik_amd/libmceik_hip.so
  for prec in ${AB_PRECS:-64}; do
    log=$O/${v}_mw${mw}_p${prec}_$r.log
    timeout -k 10 300 python3 bench.py --precision $prec --steps ${AB_STEPS:-1} --warmup 1 --no-cpu-baseline --pipes 1 \
        --max-waves $mw --f64-steps 0 > $log 2>&1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" \
        $log ${v}_mw${mw}_p$prec | tee -a $O/summary.txt
  done
done; done
for t in ${F64_TEST:-}; do
  cp mceik_amd/exp/lib_$t.so mceik_amd/libmceik_hip.so
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fsm.py tests/test_gpu_dropin.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "fp64 or f64 or double or inversion or serial or reference" > $O/tests_$t.log 2>&1 && rc=0 || rc=$?
  echo "tests $t rc=$rc" | tee -a $O/summary.txt
  [ $rc -le 1 ] || exit $rc                      # assertion failures only; a fault / abort / timeout ends the run
done
cp /tmp/keep.so mceik_amd/libmceik_hip.so
