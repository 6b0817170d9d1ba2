"""ctypes binding of libsndvae.so (include/snd_vae.h).

The HIP library is the only compute path: there is no CPU or PyTorch
fallback.  ``lib()`` raises if the shared object is missing, and ``check``
turns every negative return code into a ``SNDError`` carrying
``snd_last_error()``.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SND_LIB_PATH") or os.path.join(_HERE, "libsndvae.so")   # override: A/B builds

c_int, c_ll, c_float, c_size, c_ull = C.c_int, C.c_longlong, C.c_float, C.c_size_t, C.c_ulonglong
vp = C.c_void_p


ABI_VERSION = 17
GEN_MODES = {"sample": 0, "mean": 1, "prior": 2, "given": 3}
TOPOLOGY = {"tscale": 0, "tref": 1, "sgjoint": 2}


class SNDError(RuntimeError):
    pass


class Config(C.Structure):
    """snd_config_t"""
    _fields_ = [("n_nodes", c_int), ("f_in", c_int), ("num_feature", c_int),
                ("spatial_dim", c_int), ("h0", c_int), ("h1", c_int), ("g_hidden", c_int),
                ("latent", c_int), ("s1", c_int), ("s2", c_int), ("s3", c_int),
                ("n1", c_int), ("n2", c_int), ("beta", c_float), ("pos_weight", c_float),
                ("norm", c_float), ("dtype", c_int), ("topology", c_int), ("node_h", c_int),
                ("sampling_num", c_int), ("sg_h", c_int * 6)]


class SGGraph(C.Structure):
    """snd_sg_graph_t"""
    _fields_ = [("rowptr", vp), ("colidx", vp), ("n_rows", c_int), ("n_per_graph", c_int),
                ("edge_lr", vp), ("edge_q", vp), ("edge_rev", vp), ("node_deg", vp),
                ("node_e", vp)]


class RowTiles(C.Structure):
    """snd_row_tiles_t"""
    _fields_ = [("rows", vp), ("trp", vp), ("lcol", vp), ("ucol", vp), ("tile_rows", c_int),
                ("ustride", c_int)]


class WindowPlan(C.Structure):
    """snd_window_plan_t"""
    _fields_ = [("meta", vp), ("slots", vp), ("rows", vp), ("order", vp), ("beta", c_int)]


class Batch(C.Structure):
    """snd_batch_t"""
    _fields_ = [("rowptr", vp), ("colidx", vp), ("features", vp),
                ("feature_truth", vp), ("spatial_truth", vp), ("row_order", vp),
                ("tiles", RowTiles), ("window", WindowPlan),
                ("tree_rowptr", vp), ("tree_colidx", vp), ("rel", vp)]


class LatentReg(C.Structure):
    """snd_latent_reg_t (include/snd_vae.h)."""
    _fields_ = [(k, c_float) for k in ("w_kl", "cap_gamma", "cap_c", "w_dip", "lambda_od", "lambda_d", "w_tc")]


# name -> (restype, argtypes)
_SIGS = {
    "snd_last_error": (C.c_char_p, []),
    "snd_abi_version": (c_int, []),
    "snd_plan_set_option": (c_int, [vp, C.c_char_p, c_int]),
    "snd_dense_to_csr_workspace": (c_size, [c_int, c_int]),
    "snd_dense_to_csr": (c_int, [vp, c_int, c_int, vp, vp, c_ll, vp, vp, c_size, vp]),
    "snd_csr_spmm": (c_int, [vp, vp, c_int, vp, c_int, c_int, vp, c_int, c_int, vp, vp, vp,
                             c_int, vp, c_int, c_int, vp, vp, vp, c_int, vp]),
    "snd_csr_spmm_bf16": (c_int, [vp, vp, c_int, vp, c_int, c_int, vp, c_int, c_int, c_int, vp, vp]),
    "snd_spmm_tile_plan": (c_ll, [vp, vp, c_int, vp, c_int, vp, vp, vp, vp, C.POINTER(c_int)]),
    "snd_csr_spmm_bf16_tiled": (c_int, [vp, vp, c_int, C.POINTER(RowTiles), vp, c_int, c_int, vp,
                                        c_int, c_int, c_int, vp, vp]),
    "snd_csr_spmm_bf16_window": (c_int, [vp, vp, vp, vp, c_int, c_int, c_int, c_int, vp, c_int, c_int,
                                         vp, c_int, vp]),
    "snd_gemm": (c_int, [c_int, c_int, c_int, c_int, c_int, vp, c_int, vp, c_int, vp, c_int,
                         vp, c_int, vp]),
    "snd_conv1d_same_fwd": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, vp, vp, vp,
                                    vp, c_int, vp, c_int, c_int, vp]),
    "snd_conv1d_same_bwd_data": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, vp,
                                         c_int, c_int, vp]),
    "snd_conv1d_bwd_weight_workspace": (c_size, [c_int, c_int, c_int]),
    "snd_conv1d_same_bwd_weight": (c_int, [vp, c_int, vp, c_int, c_int, c_int, c_int, c_int,
                                           vp, vp, c_size, c_int, vp]),
    "snd_reparam_kl_blocks": (c_int, [c_int, c_int]),
    "snd_reparam_kl": (c_int, [vp, c_int, c_int, c_int, vp, c_ull, vp, vp, vp, vp, vp]),
    "snd_zzt_ce_workspace": (c_size, [c_int, c_int, c_int, c_int]),
    "snd_zzt_ce": (c_int, [vp, c_int, c_int, c_int, vp, vp, c_float, c_float, vp, vp, vp,
                           c_size, c_int, vp]),
    "snd_zzt_ce_rows_workspace": (c_size, [c_int, c_int, c_int, c_int, c_int]),
    "snd_zzt_ce_rows": (c_int, [vp, c_int, c_int, c_int, c_int, vp, vp, c_float, c_float, vp,
                                vp, vp, c_size, c_int, vp]),
    "snd_sigmoid_mse_blocks": (c_int, [c_int]),
    "snd_sigmoid_mse": (c_int, [vp, c_int, c_int, c_int, vp, vp, c_int, vp, c_int, vp, vp,
                                vp, c_int, vp, vp, vp, c_size, vp]),
    "snd_adam_tf1": (c_int, [vp, vp, vp, vp, c_ll, c_float, c_float, c_float, c_float,
                             c_float, vp, vp]),
    "snd_adam_tf1_ranges": (c_int, [vp, vp, vp, vp, vp, vp, c_int, c_float, c_float, c_float,
                                    c_float, c_float, vp, vp]),
    "snd_sg_prep": (c_int, [C.POINTER(SGGraph), vp, vp, vp]),
    "snd_sg_param_count": (c_ll, [c_int, c_int, c_int, c_int]),
    "snd_sg_workspace": (c_size, [c_int, c_int, c_int, c_int, c_int]),
    "snd_sg_layer_fwd": (c_int, [C.POINTER(SGGraph), vp, c_int, c_int, c_int, c_int, c_int, vp,
                                 c_int, vp, vp, vp, vp]),
    "snd_sg_layer_bwd": (c_int, [C.POINTER(SGGraph), vp, c_int, c_int, c_int, c_int, c_int, vp,
                                 c_int, vp, vp, vp, c_int, vp, vp, vp]),
    "snd_e2e_fwd": (c_int, [vp, c_int, c_int, c_int, vp, vp, c_int, c_int, vp, vp]),
    "snd_e2e_bwd": (c_int, [vp, c_int, c_int, c_int, vp, c_int, c_int, vp, vp, vp, vp, vp]),
    "snd_e2e_pair_fwd": (c_int, [vp, c_int, c_int, c_int, vp, vp, vp, vp]),
    "snd_e2e_pair_bwd_workspace": (c_size, [c_int, c_int, c_int]),
    "snd_e2e_pair_bwd": (c_int, [vp, vp, c_int, c_int, c_int, vp, vp, vp, vp, vp, vp, vp]),
    "snd_bn_relu_fwd": (c_int, [vp, c_ll, c_int, vp, vp, vp, vp]),
    "snd_bn_relu_bwd": (c_int, [vp, vp, c_ll, c_int, vp, vp, vp, vp, vp, vp]),
    "snd_e2e_head_ce": (c_int, [vp, vp, c_int, c_int, c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "snd_latent_reg_workspace": (c_size, [c_int, c_int]),
    "snd_latent_reg": (c_int, [vp, vp, vp, c_int, c_int, C.POINTER(LatentReg), vp, vp, vp, vp, vp]),
    "snd_bn_act_fwd": (c_int, [vp, c_int, c_ll, c_int, vp, vp, c_int, c_int, vp, c_int, vp]),
    "snd_bn_act_bwd": (c_int, [vp, c_int, vp, c_int, c_ll, c_int, vp, vp, c_int, c_int, vp, c_int, vp, vp, vp]),
    "snd_reparam_bwd": (c_int, [vp, c_int, c_int, c_int, vp, vp, vp, vp, vp, c_int, vp]),
    "snd_add_strided": (c_int, [c_ll, c_int, c_float, vp, c_int, vp, c_int, vp]),
    "snd_plan_create": (c_int, [C.POINTER(Config), c_int, C.POINTER(vp)]),
    "snd_plan_destroy": (None, [vp]),
    "snd_plan_param_count": (c_ll, [vp]),
    "snd_plan_num_blocks": (c_int, [vp]),
    "snd_plan_param_block": (c_int, [vp, c_int, C.POINTER(C.c_char_p), C.POINTER(c_ll),
                                     C.POINTER(c_ll)]),
    "snd_plan_workspace_bytes": (c_size, [vp]),
    "snd_plan_fuse_adam": (c_int, [vp, vp, vp, c_float, c_float, c_float, c_float]),
    "snd_plan_block_fused": (c_int, [vp, c_int]),
    "snd_plan_grad_event": (c_int, [vp, c_int, vp]),
    "snd_plan_grad_event_get": (c_int, [vp, c_int, C.POINTER(vp)]),
    "snd_plan_set_rng_offset": (c_int, [vp, c_ll]),
    "snd_plan_buffer": (c_int, [vp, C.c_char_p, C.POINTER(c_ll), C.POINTER(c_ll)]),
    "snd_train_step": (c_int, [vp, C.POINTER(Batch), vp, vp, vp, vp, c_ull, vp, vp, vp]),
    "snd_generate": (c_int, [vp, C.POINTER(Batch), vp, vp, c_int, vp, c_ull, vp, vp, vp]),
    "snd_plan_launch": (c_int, [vp, C.POINTER(Batch), vp, C.c_char_p, vp]),
    "snd_debug_set": (c_int, [c_int]),
}

EXPORTS = tuple(_SIGS)

_lib = None


def lib():
    """Load libsndvae.so once; raise loudly if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SNDError(f"{LIB_PATH} not built: run `python -m snd_vae_amd.build` "
                           "(no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.snd_abi_version() != ABI_VERSION:
            raise SNDError(f"{LIB_PATH}: ABI {L.snd_abi_version()} != {ABI_VERSION}; rebuild it")
        _lib = L
    return _lib


def last_error() -> str:
    return lib().snd_last_error().decode(errors="replace")


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        raise SNDError(f"{what or 'libsndvae'} failed ({rc}): {last_error()}")


def ptr(t) -> int:
    """Device pointer of a torch tensor (or 0 for None)."""
    return 0 if t is None else t.data_ptr()


def stream_ptr(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
