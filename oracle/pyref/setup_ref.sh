#!/bin/bash
# Recipe (this container only; /root/reference does not exist on the GPU box):
# copy the read-only reference Python package to a scratch dir OUTSIDE the repo, build its CPU
# neighbour op (neighbors.cpp + neighbors_cpu.cpp, g++ via torch.utils.cpp_extension) next to its
# loader, and drop in the test shims for the absent third-party deps (PyG, torch_scatter,
# torch_cluster, lightning_utilities).  Nothing from /root/reference is copied into the repo.
set -euo pipefail
DST=${TMDREF_DIR:-/tmp/tmdref}
HERE=$(cd "$(dirname "$0")" && pwd)
if [ -f "$DST/.ready" ]; then echo "$DST"; exit 0; fi
rm -rf "$DST"; mkdir -p "$DST"
cp -r /root/reference/torchmdnet "$DST/torchmdnet"
chmod -R u+w "$DST"
cp -r "$HERE/shims" "$DST/shims"
cat > "$DST/build_nb.py" <<'PY'
from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CppExtension
setup(name="tmdref_nb",
      ext_modules=[CppExtension(name="torchmdnet.neighbors.torchmdnet_neighbors",
                                sources=["torchmdnet/neighbors/neighbors.cpp",
                                         "torchmdnet/neighbors/neighbors_cpu.cpp"])],
      cmdclass={"build_ext": BuildExtension.with_options(no_python_abi_suffix=True, use_ninja=False)})
PY
(cd "$DST" && python build_nb.py build_ext --inplace > build.log 2>&1)
mkdir -p "$DST/torch_ext"
touch "$DST/.ready"
echo "$DST"
