#!/bin/bash
# Build libtmdnet_hip.so from git revision $1 into tools/_ab/lib_$1.so (A/B kernel timing with
# KBENCH_LIB=tools/_ab/lib_<rev>.so python tools/kbench.py).
set -e
rev=${1:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" torchmd-net_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/tools/_ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -shared -I"$tmp/include" \
  -I"$tmp/torchmd-net_amd/csrc" "$tmp"/torchmd-net_amd/csrc/*.hip -o "$root/tools/_ab/lib_$rev.so"
rm -rf "$tmp"
echo "$root/tools/_ab/lib_$rev.so"
