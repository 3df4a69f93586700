#!/usr/bin/env bash
# On the GPU box: bitwise GPU tests of the sampler kernel with a prebuilt
# variant mceik_amd/exp/lib_$VARIANT.so, then an interleaved A/B
# (tools/ab_bench.sh) of $AB_VARIANTS.  Outputs under gpurun_out/.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/vc
cp mceik_amd/libmceik_hip.so /tmp/keep.so
cp "mceik_amd/exp/lib_$VARIANT.so" mceik_amd/libmceik_hip.so
rc=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_mcmc.py tests/test_gpu_fsm.py \
    tests/test_gpu_interp.py tests/test_gpu_phases.py -x -q --timeout 400 --timeout-method thread \
    ${VC_K:+-k "$VC_K"} > gpurun_out/vc/tests_$VARIANT.log 2>&1 || rc=$?
cp /tmp/keep.so mceik_amd/libmceik_hip.so
[ $rc -eq 0 ] || exit $rc
bash tools/ab_bench.sh
