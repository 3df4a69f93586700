# round-4 GPU check: new tolerance / deeper-parity tests, the broken-queue test, bench with the f64 leg
set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
  tests/test_gpu_multistep.py::test_multi_step_broken_queue_is_reported \
  tests/test_gpu_tolerance.py tests/test_gpu_configs.py::test_c3_bench_production_launch_bitwise \
  tests/test_gpu_configs.py::test_c5_bench_load_launch_bitwise > gpurun_out/r04a/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r04a/bench.log 2>&1
