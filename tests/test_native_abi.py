"""CPU tests of the C-ABI boundary: the HIP library loads (no GPU needed to dlopen), exports every
symbol include/tmdnet.h declares, and the ctypes signature table matches the header."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "tmdnet.h")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    decls = {}
    for m in re.finditer(r"(?:^|\n)\s*(?:const\s+)?(?:int|size_t|char\s*\*|const char\s*\*)\s*\*?\s*(tmdnet_\w+)\s*\(([^)]*)\)\s*;",
                         txt):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        decls[m.group(1)] = args
    return decls


def test_header_declares_entry_points():
    d = _declared()
    for name in ("tmdnet_nl_build", "tmdnet_nl_backward", "tmdnet_edge_geom_fwd", "tmdnet_edge_geom_bwd",
                 "tmdnet_et_message_fwd", "tmdnet_et_message_bwd", "tmdnet_nbr_embed_fwd",
                 "tmdnet_nbr_embed_bwd", "tmdnet_tn_embed_fwd", "tmdnet_tn_embed_bwd",
                 "tmdnet_tn_message_fwd", "tmdnet_tn_message_bwd", "tmdnet_tn_node_fwd", "tmdnet_tn_node_bwd", "tmdnet_silu_fwd", "tmdnet_silu_bwd",
                 "tmdnet_atom_sum_fwd", "tmdnet_atom_sum_bwd", "tmdnet_gemm_f32", "tmdnet_pair_index",
                 "tmdnet_rbf_deriv", "tmdnet_nl_build_paired",
                 "tmdnet_edge_geom_fwd_rows",
                 "tmdnet_nl_workspace_bytes",
                 "tmdnet_build_info"):
        assert name in d, name


def test_library_exports_every_declared_symbol():
    from torchmdnet import _native
    path = _native.library_path()
    if not os.path.exists(path):
        subprocess.check_call(["make", "-C", ROOT, "-j8"], stdout=subprocess.DEVNULL)
    lib = _native.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert b"gfx950" in lib.tmdnet_build_info()


def test_ctypes_table_matches_header_arity():
    from torchmdnet import _native
    d = _declared()
    assert set(d) == set(_native.SIGNATURES)
    for name, args in d.items():
        assert len(_native.SIGNATURES[name][1]) == len(args), name


def test_library_is_gfx950_code_object():
    from torchmdnet import _native
    blob = open(_native.library_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_product_has_no_cpu_fallback():
    import torch
    from torchmdnet.neighbors import get_neighbor_pairs_kernel
    pos = torch.zeros(4, 3)
    batch = torch.zeros(4, dtype=torch.long)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        get_neighbor_pairs_kernel("brute", pos, batch, torch.empty((0, 0)), False, 0.0, 1.0, 16, True, True)


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "torchmd-net_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r"#.*", "", src).replace("Oracle", ""), f
