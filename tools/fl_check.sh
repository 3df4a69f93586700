set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fl
cp mceik_amd/libmceik_hip.so /tmp/keep.so
cp mceik_amd/exp/lib_fl.so mceik_amd/libmceik_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_mcmc.py -x -q --timeout 300 --timeout-method thread -k "c3_sampler_forward or c3_mcmc_two or c2_workload or pipes or accept_sequence" > gpurun_out/fl/tests.log 2>&1 || { cp /tmp/keep.so mceik_amd/libmceik_hip.so; exit 1; }
cp /tmp/keep.so mceik_amd/libmceik_hip.so
AB_VARIANTS="base2 fl" AB_ROUNDS=2 AB_ARGS="--steps 2 --warmup 1 --pipes 1" bash tools/ab_bench.sh
