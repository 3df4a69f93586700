# full GPU suite + smoke + default bench (round 4)
set -o pipefail
out=gpurun_out/${1:-r04b}
mkdir -p $out
timeout -k 10 120 ./tools/sqrt_dir_probe > $out/sqrt_dir_probe.log 2>&1 && \
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1
