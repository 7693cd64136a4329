"""Loader for the C-ABI HIP library ``lib/libtmdnet_hip.so`` (declared in ``include/tmdnet.h``).

The library is bound with ctypes AFTER torch is imported, so its ``libamdhip64.so.7`` dependency
resolves to the HIP runtime torch already loaded (one runtime, one set of streams).  Every hot-path
entry point of this package goes through here; if the library is missing or the device is not a ROCm
GPU the call raises -- there is no CPU or eager-PyTorch fallback on the product path.
"""
import ctypes
import os

import torch

# TMDNET_LIB=debug selects the build with the CSR kernels' index-range checks (`make debug`)
_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                         "libtmdnet_hip_debug.so" if os.environ.get("TMDNET_LIB") == "debug" else "libtmdnet_hip.so")

F32, F64 = 0, 1
NL_BRUTE, NL_SHARED, NL_CELL = 0, 1, 2
RBF_EXPNORM, RBF_GAUSS = 0, 1
ACC_VEC_RESIDUAL, ACC_EDGE = 1, 2
ACC_GRADS = 32
ET_V_PLANAR = 4
BWD2_ACC_EDGE, BWD2_ACC_GVEC = 8, 16
ET_TWO_PASS = 64

_STATUS = {1: "bad argument", 2: "unsupported configuration", 3: "kernel launch failed",
           4: "workspace too small"}

P = ctypes.c_void_p
I = ctypes.c_int
D = ctypes.c_double
SZ = ctypes.c_size_t

# name -> (restype, argtypes); must match include/tmdnet.h exactly (tests check the exports)
SIGNATURES = {
    "tmdnet_nl_workspace_bytes": (SZ, [I, I, P, D]),
    "tmdnet_nl_build": (I, [I, I, P, P, I, P, I, D, D, I, I, I, P, P, P, P, P, P, I, P, SZ, P]),
    "tmdnet_nl_build_paired": (I, [I, I, P, P, I, P, I, D, D, I, I, I, P, P, P, P, P, P, I, P, SZ, P, P, I, P]),
    "tmdnet_nl_backward": (I, [I, I, P, P, I, P, P, P, P, P, P]),
    "tmdnet_nl_backward_multi": (I, [I, I, P, P, I, P, P, P, P, P, P, P]),
    "tmdnet_nl_backward2": (I, [I, I, P, P, P, I, P, P, P, P, P, P, P, P]),
    "tmdnet_nl_backward_edges": (I, [I, I, P, I, P, P, P, P, P, P]),
    "tmdnet_edge_geom_fwd": (I, [I, I, I, I, P, P, P, P, P, P, D, D, P, P, P, P]),
    "tmdnet_edge_geom_fwd_rows": (I, [I, I, I, I, P, P, P, P, P, P, D, D, P, P, P, P, I, P, P]),
    "tmdnet_edge_geom_fwd_rows2": (I, [I, I, I, I, P, P, P, P, P, P, D, D, P, P, P, P, I, P, P, P]),
    "tmdnet_edge_geom_bwd": (I, [I, I, I, I, P, P, P, P, P, P, D, D, P, P, P, P, P, P]),
    "tmdnet_edge_geom_bwd_multi": (I, [I, I, I, I, P, P, P, P, P, P, D, D, P, P, P, P, P, P, P, P, P, P]),
    "tmdnet_edge_geom_bwd2": (I, [I, I, I, I, P, P, P, P, P, P, D, D, P, P, P, P, P, P, P, P, P, P, P]),
    "tmdnet_et_message_fwd": (I, [I, I, I, I, P, P, I, P, I, P, I, P, I, P, P, I, P, I, P, P, P, P, I, P, P,
                                  P]),
    "tmdnet_et_message_bwd": (I, [I, I, I, I, P, P, I, P, I, P, I, P, I, P, P, I, P, I, P, P, P, P,
                                  P, P, P, P, P, P, P, P, P, P, P, I, P, P, P]),
    "tmdnet_rbf_deriv": (I, [I, I, I, P, P, P, D, D, P, I, P, P]),
    "tmdnet_pair_index_workspace_bytes": (SZ, [I]),
    "tmdnet_pair_index": (I, [I, P, P, P, P, I, P, I, P, P, I, P, SZ, P]),
    "tmdnet_et_message_bwd2": (I, [I, I, I, I, P, P, I, P, I, P, I, P, I, P, P, I, P, I, P, P, P, P,
                                   P, P, P, P, P, I, P, I, P, P, P, P, P, P, P, P, P, P, P, P, I, P]),
    "tmdnet_et_message_bwd2_ex": (I, [I, I, I, I, P, P, P, I, P, I, P, I, P, I, P, P, I, P, I, P, P, P, P,
                                      P, I, P, I, P, I, P, P, I, P, I, P, P,
                                      P, P, P, I, P, I, P, I, P, P, I, P, I, P, P, P, P, P, I, P]),
    "tmdnet_et_epilogue_fwd": (I, [I, I, I, P, P, P, P, P, P, P, P]),
    "tmdnet_et_epilogue_bwd": (I, [I, I, I, P, P, P, P, P, P, P]),
    "tmdnet_et_epilogue_bwd_acc": (I, [I, I, I, P, P, P, P, P, P, I, P]),
    "tmdnet_et_epilogue_ln_fwd": (I, [I, I, I, P, P, P, P, P, P, P, D, P, P, P, P, P, P]),
    "tmdnet_ln_bwd_epilogue": (I, [I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "tmdnet_ln_bwd_epilogue_w": (I, [I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, P]),
    "tmdnet_et_oproj_epilogue_f32": (I, [I, I] + [P] * 11),
    "tmdnet_et_ln_mix_f32": (I, [I, I, P, P, P, D, P, P, I, P, P, P, P, P, P, I, P, P]),
    "tmdnet_et_lnbwd_oproj_f32": (I, [I, I] + [P] * 15),
    "tmdnet_et_adjoint_epi_ln": (I, [I, I, I] + [P] * 21),
    "tmdnet_et_adjoint_epi_ln2": (I, [I, I, I] + [P] * 22),
    "tmdnet_eq_head_fwd": (I, [I, I, I, P, P, P, P, P, P, P]),
    "tmdnet_eq_head_bwd": (I, [I, I, I, P, P, P, P, P, P]),
    "tmdnet_eq_head_bwd_weights": (I, [I, I, I, P, P, P, P, P, P, P, P]),
    "tmdnet_eq_head_hvp": (I, [I, I, I, P, P, P, P, P, P, P, P, P, P, P]),
    "tmdnet_nbr_embed_fwd": (I, [I, I, I, P, P, I, P, I, P, I, P, P, I, P, P, P]),
    "tmdnet_nbr_embed_bwd": (I, [I, I, I, P, P, I, P, I, P, I, P, P, I, P, P, P, P]),
    "tmdnet_nbr_embed_bwd2": (I, [I, I, I, P, P, P, I, P, I, P, I, P, P, I, P, P, P, P, P, P, P, P]),
    "tmdnet_tn_embed_fwd": (I, [I, I, I, P, P, I, D, P, I, P, P, P, I, P, P, P, P]),
    "tmdnet_tn_embed_bwd": (I, [I, I, I, P, P, I, D, P, I, P, P, P, I, P, P, P, P, P, P, P, P, P]),
    "tmdnet_tn_embed_bwd2": (I, [I, I, I, P, P, I, D, P, I, P, P, P, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P,
                                 P]),
    "tmdnet_tn_message_fwd": (I, [I, I, I, P, P, I, D, P, I, P, I, P, P, P]),
    "tmdnet_tn_message_bwd": (I, [I, I, I, P, P, I, D, P, I, P, I, P, P, P, P, P]),
    "tmdnet_tn_message_bwd_add": (I, [I, I, I, P, P, I, D, P, I, P, I, P, P, P, P, P, P]),
    "tmdnet_tn_message_fwd_pairs": (I, [I, I, I, P, P, I, D, P, I, P, P, I, P, P, P]),
    "tmdnet_tn_message_bwd_pairs": (I, [I, I, I, P, P, I, D, P, I, P, P, I, P, I, P, P, P, P, P, P]),
    "tmdnet_tn_node_fwd": (I, [I, I, I, I, P, P, P, P]),
    "tmdnet_tn_node_bwd": (I, [I, I, I, I, P, P, P, P, P, P, P]),
    "tmdnet_tn_node_bwd2": (I, [I, I, I, I, P, P, P, P, P, P, P, P, P]),
    "tmdnet_silu_fwd": (I, [I, I, I, P, I, P, P, P]),
    "tmdnet_silu_bwd": (I, [I, I, I, P, I, P, P, I, P, P, P]),
    "tmdnet_mlp2_up": (I, [I, I, I, P, I, P, P, I, P, P, P, P, P, P, P, P]),
    "tmdnet_mlp2_down": (I, [I, I, I, P, I, P, P, P, P]),
    "tmdnet_atom_sum_fwd": (I, [I, I, I, P, P, P, P, P, P]),
    "tmdnet_atom_sum_bwd": (I, [I, I, I, P, P, P, P, P]),
    "tmdnet_dot_sum_fwd": (I, [I, I, I, P, I, P, P, I, P, P, P, P, P]),
    "tmdnet_dot_sum_bwd": (I, [I, I, I, P, P, I, P, P, P, P]),
    "tmdnet_dot_sum_fwd_atoms": (I, [I, I, I, P, I, P, P, I, P, P, P, P, P, P]),
    "tmdnet_layernorm_fwd_f32": (I, [I, I, P, I, P, P, D, P, I, P, P, P]),
    "tmdnet_layernorm_bwd_f32": (I, [I, I, P, I, P, P, P, P, I, P, I, P]),
    "tmdnet_layernorm_bwd2_f32": (I, [I, I, P, I, P, P, P, P, I, P, P, P, P, P, P, P]),
    "tmdnet_layernorm_wgrad_workspace_bytes": (SZ, [I, I]),
    "tmdnet_layernorm_wgrad_f32": (I, [I, I, P, I, P, P, P, I, P, P, P, SZ, P]),
    "tmdnet_gemm_f32": (I, [I, P, P, P]),
    "tmdnet_gemm_ex_f32": (I, [I, P, P, P]),
    "tmdnet_gemm_tn_f32": (I, [I, P, P, P]),
    "tmdnet_gemm_tn_workspace_bytes": (ctypes.c_size_t, [I, P]),
    "tmdnet_gemm_tn_f32_ws": (I, [I, P, P, P, ctypes.c_size_t, P]),
    "tmdnet_gemm_tn_rows_f32_ws": (I, [I, P, P, P, ctypes.c_size_t, P]),
    "tmdnet_embedding_bwd_f32": (I, [I, I, I, P, I, P, P, P, I, P]),
    "tmdnet_embedding_fwd_f32": (I, [I, I, I, P, I, P, P, P, P, P]),
    "tmdnet_proj_split_f32": (I, [I, I, P, I, P, P]),
    "tmdnet_split_t_f32": (I, [I, I, P, I, P, P]),
    "tmdnet_gemm_x3_f32": (I, [I, I, I, P, I, P, P, P, I, I, P]),
    "tmdnet_gemm_x3_ex_f32": (I, [I, I, I, P, I, P, P, P, I, I, I, P, P, P, I, P]),
    "tmdnet_gemm_x3w_f32": (I, [I, I, I, P, I, P, I, I, P, P, I, I, I, P, P, P, I, P]),
    "tmdnet_fep_image_bytes": (SZ, [I, I]),
    "tmdnet_fep_split_f32": (I, [I, I, P, I, P, P, P, P, P]),
    "tmdnet_et_fused_bwd_f32": (I, [I, I, I, I, P, P, I, P, I, P, I, P, I, P, P, P, P, P, P, ctypes.c_longlong, P, P, P,
                                    P, P, P, P, P, P, P, P, P, I, P, SZ, P]),
    "tmdnet_et_fused_bwd_workspace_bytes": (SZ, [I]),
    "tmdnet_et_fused_fwd_f32": (I, [I, I, I, I, P, P, I, P, I, P, I, P, I, P, P, P, P, P, ctypes.c_longlong, P, P, P, P, P,
                                    I, P]),
    "tmdnet_nbr_fused_fwd_f32": (I, [I, I, I, P, P, I, P, I, P, P, P, ctypes.c_longlong, P, P, P, P, I, P, P, P]),
    "tmdnet_nbr_fused_bwd_f32": (I, [I, I, I, P, P, I, P, I, P, P, P, P, ctypes.c_longlong, P, P, P, P, I, P, P, I,
                                     P]),
    "tmdnet_eq_head_x3_f32": (I, [I, I, P, P, P, P, P, P, P, P, P]),
    "tmdnet_eq_head_x3_pieces_bytes": (SZ, [I]),
    "tmdnet_eq_head_x3_split_f32": (I, [I, P, P, P]),
    "tmdnet_fep_frags_bytes": (SZ, [ctypes.c_longlong, I]),
    "tmdnet_fep_frags_f32": (I, [ctypes.c_longlong, I, P, P, P, D, D, I, P, P, P]),
    "tmdnet_proj_f32": (I, [I, I, I, P, I, P, ctypes.c_longlong, P, P, I, P]),
    "tmdnet_mse2_fwd": (I, [I, I, P, P, D, I, P, P, D, P, P]),
    "tmdnet_mse2_bwd": (I, [I, I, P, P, D, I, P, P, D, P, P, P, P]),
    "tmdnet_build_info": (ctypes.c_char_p, []),
    "tmdnet_set_tuning": (I, [I, I]),
}

_lib = None
_torch_ops_loaded = False
_TORCH_OPS_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libtmdnet_torch.so")


def load_torch_ops():
    """Register the dispatcher operators of ``lib/libtmdnet_torch.so`` (csrc/torch_ops.cpp):
    ``torchmdnet_neighbors::get_neighbor_pairs`` (the reference schema) and the ``tmdnet::*`` ops of
    the TorchScript model path.  Raises if the library is absent (no fallback)."""
    global _torch_ops_loaded
    if _torch_ops_loaded:
        return
    if not os.path.exists(_TORCH_OPS_PATH):
        raise RuntimeError(f"torchmd-net_amd: operator library not found at {_TORCH_OPS_PATH}; run `make`")
    torch.ops.load_library(_TORCH_OPS_PATH)
    _torch_ops_loaded = True


def invalidate_stack_cache():
    """No-op kept for compatibility: the C++ ``tmdnet::et_stack`` operator used to cache packed weights keyed
    on parameter versions (which fused optimizers and ``p.data`` writes do not bump); it now takes them as
    views of the parameters' own storage on every call (torch_ops.cpp ``pack_stack``), so nothing can go
    stale."""
    if _torch_ops_loaded:
        torch.ops.tmdnet.et_stack_invalidate()


def library_path():
    return _LIB_PATH


def load(required=True):
    """Load and return the ctypes handle (raises if the library is absent and ``required``)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        if required:
            raise RuntimeError(
                f"torchmd-net_amd: HIP library not found at {_LIB_PATH}; run `make` (or "
                "__graft_entry__.build()) -- there is no CPU fallback for the hot path")
        return None
    lib = ctypes.CDLL(_LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"torchmd-net_amd: {what} failed: {_STATUS.get(rc, rc)}")


def require_gpu(t, what):
    if not t.is_cuda:
        raise RuntimeError(
            f"torchmd-net_amd: {what} runs only on a ROCm GPU (got a {t.device} tensor); this "
            "package has no CPU implementation of the hot path")


def dtype_code(dtype):
    if dtype == torch.float32:
        return F32
    if dtype == torch.float64:
        return F64
    raise RuntimeError(f"torchmd-net_amd: unsupported floating type {dtype} (float32/float64)")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
