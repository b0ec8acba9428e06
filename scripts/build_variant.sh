#!/bin/bash
# Build libsentinel_gpu.so from a git ref (or the working tree: ref "wt") into build/ab/<name>.so, for A/B runs
# on one box through SG_LIB_PATH:  scripts/build_variant.sh <name> <ref> [extra hipcc flags]
set -e
name=$1 ref=$2 extra=$3
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=/tmp/ab_$name
rm -rf "$tmp"; mkdir -p "$tmp"
if [ "$ref" = wt ]; then
  cp -r "$root/sentinel_amd" "$root/include" "$tmp/"
else
  (cd "$root" && git archive "$ref" sentinel_amd include) | tar -x -C "$tmp"
fi
mkdir -p "$root/build/ab"
make -s -j8 -C "$tmp/sentinel_amd/csrc" OUT="$root/build/ab/$name.so" BUILD="$tmp/build" HOSTLIB="$tmp/host.so" \
  COMMON="-O3 -std=c++17 -fPIC -fwrapv -ffp-contract=off -Wall -Wno-unused-result $extra" "$root/build/ab/$name.so"
echo "built build/ab/$name.so"
