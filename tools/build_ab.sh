#!/usr/bin/env bash
# Builds ab/libpbx_ab.so (git-ignored, outside the product lib/) from git revision $1 (default HEAD) for
# same-box A/B timing: PBX_AB_LIBRARY=<path> python tools/run_leg.py ...
set -euo pipefail
rev=${1:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
git -C "$root" archive "$rev" pynbody-extras_amd/csrc include | tar -x -C "$tmp"
make -s -j8 -C "$tmp/pynbody-extras_amd/csrc" OUT="$root/ab/libpbx_ab.so"
echo "built libpbx_ab.so from $(git -C "$root" rev-parse --short "$rev")"
