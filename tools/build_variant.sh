#!/usr/bin/env bash
# Builds ab/<NAME>.so (git-ignored, outside the product lib/) from the WORKING
# TREE's sources with extra compiler flags, for same-box A/B timing of a
# compile-time constant: tools/build_variant.sh NAME -DPBX_SYM_DPP_MASK=0x0F
# then PBX_AB_LIBRARY=ab/NAME.so python bench.py ...
set -euo pipefail
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
mkdir -p "$tmp/pynbody-extras_amd" "$root/ab"
cp -r "$root/include" "$tmp/"
cp -r "$root/pynbody-extras_amd/csrc" "$tmp/pynbody-extras_amd/"
rm -rf "$tmp/pynbody-extras_amd/csrc/build"
make -s -j8 -C "$tmp/pynbody-extras_amd/csrc" OUT="$root/ab/$name.so" \
  CXXFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-gpu-rdc -I../../include $*"
echo "built ab/$name.so with $*"
