#!/usr/bin/env bash
# Builds ab/libpbx_<tag>.so (git-ignored) from the working tree with extra
# compile flags (timing diagnostics): tools/build_diag.sh TAG -DPBX_DIAG_...
set -euo pipefail
tag=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
mkdir -p "$tmp/pynbody-extras_amd"
cp -r "$root/pynbody-extras_amd/csrc" "$tmp/pynbody-extras_amd/"
rm -rf "$tmp/pynbody-extras_amd/csrc/build"
cp -r "$root/include" "$tmp/"
make -s -j8 -C "$tmp/pynbody-extras_amd/csrc" OUT="$root/ab/libpbx_$tag.so" \
  CXXFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-gpu-rdc -I../../include $*"
echo "built libpbx_$tag.so ($*)"
