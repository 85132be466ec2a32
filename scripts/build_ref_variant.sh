#!/bin/bash
# Build libbdx_hip_<name>.so from the HIP sources of git revision <rev> (for
# same-box A/B runs: BDX_HIP_LIB=libbdx_hip_<name>.so python bench.py ...).
#   scripts/build_ref_variant.sh <rev> <name>
set -e
rev=${1:-HEAD}; name=${2:-head}
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" benchmark_dolfinx_amd | tar -x -C "$tmp"
(cd "$tmp" && python -m benchmark_dolfinx_amd.ops.build --hip -j 8 > /dev/null)
cp "$tmp/benchmark_dolfinx_amd/ops/libbdx_hip.so" "$root/benchmark_dolfinx_amd/ops/libbdx_hip_$name.so"
rm -rf "$tmp"
echo "built benchmark_dolfinx_amd/ops/libbdx_hip_$name.so from $rev"
