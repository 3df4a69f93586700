# fp64 compact-layout A/B (f64d: v31, 6 waves/CU; f64g: compact LDS, 8 waves/CU) + the full GPU suite on the in-tree build
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
F64_OUT=r04_cmp F64_VARIANTS="f64d f64g" bash tools/f64_ab.sh
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04_cmp/gpu_tests.log 2>&1
