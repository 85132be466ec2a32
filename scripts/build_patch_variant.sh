#!/bin/bash
# Build libbdx_hip_<name>.so from the working tree's HIP sources with one or
# more literal text substitutions applied to a scratch copy (same-box A/B of
# a kernel variant without adding switches to the production headers).
#   scripts/build_patch_variant.sh <name> <file> <old> <new> [<file> <old> <new> ...]
set -e
name=$1; shift
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d)
cp -r "$root/benchmark_dolfinx_amd" "$tmp/"
rm -f "$tmp"/benchmark_dolfinx_amd/ops/*.so "$tmp"/benchmark_dolfinx_amd/ops/*.sha1
while [ $# -ge 3 ]; do
  python3 - "$tmp/benchmark_dolfinx_amd/csrc/hip/$1" "$2" "$3" <<'PY'
import sys
p, old, new = sys.argv[1:4]
s = open(p).read()
assert s.count(old) == 1, f"{p}: {old!r} occurs {s.count(old)} times"
open(p, "w").write(s.replace(old, new))
PY
  shift 3
done
(cd "$tmp" && python -m benchmark_dolfinx_amd.ops.build --hip -j 8 > /dev/null)
cp "$tmp/benchmark_dolfinx_amd/ops/libbdx_hip.so" "$root/benchmark_dolfinx_amd/ops/libbdx_hip_$name.so"
rm -rf "$tmp"
echo "built benchmark_dolfinx_amd/ops/libbdx_hip_$name.so"
