"""Compile the REFERENCE CPU neighbour op (neighbors.cpp + neighbors_cpu.cpp, read in place from
/root/reference/torchmdnet/neighbors/, never copied) into oracle/_ref/ with g++ via
torch.utils.cpp_extension.  Test infrastructure only; /root/reference exists only in the build
container, so on the GPU box this is skipped and tests fall back to the committed fixtures."""
import os
import sys

SRC = "/root/reference/torchmdnet/neighbors"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref")


def main():
    if not os.path.isdir(SRC):
        print("reference sources absent; skipping oracle/_ref")
        return 0
    os.makedirs(OUT, exist_ok=True)
    from torch.utils.cpp_extension import load
    load(name="tmdref_neighbors", sources=[os.path.join(SRC, "neighbors.cpp"), os.path.join(SRC, "neighbors_cpu.cpp")],
         build_directory=OUT, is_python_module=False, verbose=False)
    print("built", OUT)
    return 0


if __name__ == "__main__":
    sys.exit(main())
