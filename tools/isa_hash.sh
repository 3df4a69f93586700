#!/usr/bin/env bash
# sha256 of the gfx950 assembly of every kernel source, compiled with the
# library's flags (mceik_amd/Makefile FLAGS) plus any extra flags given.
# A refactor that must not change the default build's code objects compares
# this output before and after.   usage: tools/isa_hash.sh [extra flags...]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT/mceik_amd"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wall -Wno-unused-function -Wno-unused-value"
T=$(mktemp -d /tmp/isa_XXXX)
for f in fsm_kernel fsm16_kernel fsm_single mcmc_kernels capi comm; do
  ( /opt/rocm/bin/hipcc $FLAGS "$@" --cuda-device-only -S csrc/$f.hip -o "$T/$f.s" 2>/dev/null
    # drop the compiler's ident/path lines, keep the ISA and kernel metadata
    # and the per-translation-unit id (__hip_cuid_<hash of the path and source>)
    grep -v -E '^\s*\.(ident|file)\b' "$T/$f.s" | sed -E 's/__hip_cuid_[0-9a-f]+/__hip_cuid/g' | sha256sum |
        sed "s|-|$f|" ) &
done
wait
rm -rf "$T"
