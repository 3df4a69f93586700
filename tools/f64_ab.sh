set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/${F64_OUT:-f64e}
cp mceik_amd/libmceik_hip.so /tmp/keep.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_fsm.py -x -q --timeout 250 --timeout-method thread -k "fp64 or inversion" > gpurun_out/${F64_OUT:-f64e}/tests.log 2>&1
for r in 1 2; do for v in ${F64_VARIANTS:-f64br f64sel}; do
  cp mceik_amd/exp/lib_$v.so mceik_amd/libmceik_hip.so
  timeout -k 10 300 python3 bench.py --precision 64 --steps 1 --warmup 1 --no-cpu-baseline --pipes 1 > gpurun_out/${F64_OUT:-f64e}/${v}_$r.log 2>&1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" gpurun_out/${F64_OUT:-f64e}/${v}_$r.log $v | tee -a gpurun_out/${F64_OUT:-f64e}/summary.txt
done; done
cp /tmp/keep.so mceik_amd/libmceik_hip.so
