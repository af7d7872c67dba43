"""ctypes binding of libray_amd_hip.so (the hand-written CDNA4 kernels).

The library is built in-tree by ``ray_amd._native.build``. On a machine with a
GPU the HIP path is mandatory: if the library is missing or fails to load,
``lib()`` raises instead of silently falling back to eager PyTorch. CPU tensors
use the plain-PyTorch reference implementations in ``ray_amd.ops.reference``
(that is also what the numerics tests compare the kernels against).
"""

from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_native", "libray_amd_hip.so")

_lib = None
_lock = threading.Lock()

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_long = ctypes.c_long
c_float = ctypes.c_float
c_double = ctypes.c_double
c_size_t = ctypes.c_size_t

_SIGS = {
    "ra_layernorm_fwd": [c_void_p] * 6 + [c_int, c_int, c_float, c_void_p],
    "ra_layernorm_bwd_parts": [c_int],
    "ra_layernorm_bwd": [c_void_p] * 11 + [c_int, c_int, c_int, c_void_p],
    "ra_residual_layernorm_fwd": [c_void_p] * 9 + [c_int, c_int, c_float, c_void_p],
    "ra_colsum": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "ra_layernorm_bwd_work": [c_int, c_int],
    "ra_colsum_work": [c_int, c_int],
    "ra_colsum_parts": [c_int, c_int],
    "ra_bias_gelu_fwd": [c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p],
    "ra_bias_gelu_bwd": [c_void_p] * 6 + [c_int, c_int, c_int, c_void_p],
    "ra_colsum_bf16": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "ra_splitk_accum": [c_void_p, c_int, c_long, c_void_p, c_int, c_void_p],
    "ra_transpose_bf16": [c_void_p, c_void_p, c_int, c_int, c_void_p],
    "ra_wgrad": [c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int, c_int, c_void_p,
                 c_void_p, c_int, c_void_p],
    "ra_wgrad_splits": [c_int, c_int, c_int],
    "ra_bias_residual": [c_void_p] * 4 + [c_long, c_int, c_void_p],
    "ra_xent_fwd": [c_void_p] * 4 + [c_int, c_int, c_int, c_long, c_void_p],
    "ra_xent_bwd": [c_void_p] * 4 + [c_float, c_void_p, c_int, c_int, c_int, c_long, c_void_p],
    "ra_norm_parts": [],
    "ra_grad_clip": [c_void_p, c_long, c_int, c_float, c_float, c_void_p, c_void_p, c_void_p,
                     c_void_p],
    "ra_adamw_flat": [c_void_p] * 5 + [c_long, c_long] + [c_float] * 5 + [c_int, c_void_p,
                                                                            c_int, c_void_p],
    "ra_adamw_flat_wt": [c_void_p] * 6 + [c_long, c_long, c_long, c_void_p, c_int]
                        + [c_float] * 5 + [c_int, c_void_p, c_int, c_void_p, c_void_p],
    "ra_wt_table_bytes": [],
    "ra_wt_max_segments": [],
    "ra_adamw_flat_dev": [c_void_p] * 5 + [c_long, c_long] + [c_float] * 5 +
    [c_int, c_void_p, c_int, c_void_p, c_void_p],
    "ra_scaled_accum": [c_void_p, c_void_p, c_long, c_int, c_void_p, c_void_p],
    "ra_scale_bf16": [c_void_p, c_long, c_void_p, c_void_p],
    "ra_xent_fused": [c_void_p] * 4 + [c_int, c_int, c_int, c_long, c_void_p],
    "ra_adamw_f32": [c_void_p] * 4 + [c_long, c_long] + [c_float] * 5 + [c_int, c_void_p,
                                                                           c_void_p],
    "ra_sgd_flat": [c_void_p] * 4 + [c_long, c_float, c_float, c_float, c_void_p, c_void_p],
    "ra_gae": [c_void_p] * 6 + [c_int, c_int, c_float, c_float, c_void_p],
    "ra_vtrace": [c_void_p] * 7 + [c_int, c_int] + [c_float] * 4 + [c_void_p],
    "ra_ppo_loss": [c_void_p] * 10 + [c_int, c_int] + [c_float] * 5 + [c_int, c_void_p],
    "ra_ppo_loss_packed": [c_void_p, c_void_p, c_void_p, c_int, c_int] + [c_void_p] * 4
                          + [c_int, c_int] + [c_float] * 5 + [c_void_p, c_int, c_float, c_void_p],
    "ra_scale_to_bf16": [c_void_p, c_long, c_void_p, c_void_p, c_void_p],
    "ra_ppo_heads_fwd": [c_void_p, c_int] + [c_void_p] * 5 + [c_int, c_int] + [c_void_p] * 3
                        + [c_int, c_int] + [c_float] * 5 + [c_void_p, c_float, c_void_p],
    "ra_ppo_heads_work": [c_int, c_int],
    "ra_ppo_heads_bwd": [c_void_p, c_int] + [c_void_p] * 10 + [c_int, c_int, c_int, c_void_p],
    "ra_bias_relu_fwd": [c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p],
    "ra_relu_bwd_work": [c_int, c_int],
    "ra_relu_bwd_bias": [c_void_p] * 5 + [c_int, c_int, c_int, c_void_p],
    "ra_obsnorm_parts": [c_int],
    "ra_obsnorm_update": [c_void_p, c_int, c_int, c_double, c_void_p, c_void_p, c_void_p,
                          c_void_p],
    "ra_obsnorm_apply": [c_void_p] * 4 + [c_long, c_int, c_double, c_float, c_float, c_void_p],
    "ra_lt_num_cands": [c_int, c_int] + [c_long] * 6,
    "ra_lt_release_stream": [c_void_p],
    "ra_embed_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                     c_void_p],
    "ra_lt_num_streams": [],
    "ra_lt_set_choice": [c_int, c_int] + [c_long] * 6 + [c_int],
    "ra_lt_gemm": [c_int, c_int, c_long, c_long, c_long, c_void_p, c_long, c_void_p, c_long,
                   c_void_p, c_long, c_float, c_float, c_void_p],
    "ra_lt_tune": [c_int, c_int, c_long, c_long, c_long, c_void_p, c_long, c_void_p, c_long,
                   c_void_p, c_long, c_int, c_void_p, c_int, c_long, c_long, c_long, c_void_p],
    "ra_lt_gemm_batched": [c_int, c_int, c_long, c_long, c_long, c_void_p, c_long, c_long,
                           c_void_p, c_long, c_long, c_void_p, c_long, c_long, c_int, c_float,
                           c_float, c_void_p],
    "ra_lt_ep_num_cands": [c_int, c_int] + [c_long] * 6 + [c_int, c_long],
    "ra_lt_ep_set_choice": [c_int, c_int] + [c_long] * 6 + [c_int, c_long, c_int],
    "ra_lt_gemm_ep": [c_int, c_int, c_long, c_long, c_long, c_void_p, c_long, c_void_p, c_long,
                      c_void_p, c_long, c_int, c_void_p, c_void_p, c_long, c_int, c_void_p],
    "ra_lt_num_cands_batched": [c_int, c_int] + [c_long] * 6 + [c_int, c_long, c_long, c_long],
    "ra_lt_set_choice_batched": [c_int, c_int] + [c_long] * 6 + [c_int, c_long, c_long, c_long,
                                                                  c_int],
    "ra_lt_choice_name": [c_int, c_int] + [c_long] * 6 + [c_int, c_long, c_long, c_long,
                                                           ctypes.c_char_p, c_int],
    "ra_lt_allow_streamk": [c_int],
    "ra_lt_choice_is_streamk": [c_int, c_int] + [c_long] * 6 + [c_int, c_long, c_long, c_long],
    "ra_image_normalize": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                           c_int, c_void_p],
    "ra_resize_bilinear": [c_void_p, c_void_p] + [c_int] * 6 + [c_void_p],
    "ra_cast_scale_u8": [c_void_p, c_void_p, c_long, c_float, c_void_p],
    "ra_gather_cast_u8": [c_void_p, c_void_p, c_void_p, c_long, c_long, c_float, c_void_p],
    "ra_conv_supported": [c_int] * 6,
    "ra_conv_fwd": [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p] + [c_int] * 8
                   + [c_float, c_int, c_void_p],
    "ra_conv_wgrad_work": [c_int] * 8,
    "ra_conv_dgrad_supported": [c_int] * 5,
    "ra_conv_dgrad": [c_void_p] * 3 + [c_int] * 8 + [c_void_p],
    "ra_conv_wgrad": [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_long, c_void_p, c_int]
                     + [c_int] * 8 + [c_float, c_void_p],
    "ra_attn_fwd": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                    c_void_p],
    "ra_attn_bwd": [c_void_p] * 6 + [c_int, c_int, c_int, c_int, c_float, c_void_p],
    "ra_gemm_nt": [c_void_p, c_long, c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int,
                   c_int, c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_int, c_int,
                   c_void_p],
    "ra_gemm_dgelu_work": [c_int, c_int],
    "ra_arena_alloc": [c_int, c_size_t, ctypes.POINTER(c_void_p), c_void_p],
    "ra_ipc_handle_size": [],
    "ra_arena_open": [c_int, c_void_p, ctypes.POINTER(c_void_p)],
    "ra_arena_close": [c_void_p],
    "ra_arena_free": [c_void_p],
    "ra_copy_async": [c_void_p, c_void_p, c_size_t, c_void_p],
    "ra_stream_sync": [c_void_p],
    "ra_device_count": [ctypes.POINTER(c_int)],
    "ra_host_register": [c_void_p, c_size_t],
    "ra_host_unregister": [c_void_p],
}




class HipKernelError(RuntimeError):
    pass


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            # Build on first use (cheap: hipcc cross-compiles in seconds).
            from ray_amd._native.build import build_hip

            build_hip()
        L = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = c_long if name.endswith("_work") else c_int
        _lib = L
    return _lib


def check(rc: int, name: str = "kernel") -> None:
    if rc != 0:
        raise HipKernelError(f"{name} failed with hipError {rc}")


def stream_ptr(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()
