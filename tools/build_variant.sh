#!/usr/bin/env bash
# Builds an experimental libmceik_hip.so with extra compiler flags into
# mceik_amd/exp/lib_<name>.so (for tools/ab_bench.sh / tools/pmc_ab.sh).
# usage: tools/build_variant.sh <name> [extra hipcc flags...]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
B=$(mktemp -d /tmp/variant_XXXX)
cd "$ROOT/mceik_amd"
make -s -j8 BUILD_DIR="$B" EXTRA="$*" OUT="$B/lib.so" "$B/lib.so"
mkdir -p exp
cp "$B/lib.so" "exp/lib_$NAME.so"
rm -rf "$B"
echo "exp/lib_$NAME.so"
