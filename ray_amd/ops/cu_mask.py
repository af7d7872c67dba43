"""HIP streams restricted to a subset of the GPU's compute units (hipExtStreamCreateWithCUMask).

Experiment knob for the two-stream GPT-2 step: the weight-gradient side stream and the main
stream can be given disjoint CU sets (RAY_AMD_SIDE_CUS / RAY_AMD_MAIN_CUS), so that the main
stream's persistent GEMMs (one workgroup per CU) never share a CU with a weight-gradient
workgroup (profiles/r5/r5e: a dgrad GEMM runs 2-5x slower when they do)."""

from __future__ import annotations

import ctypes

import torch

_hip = None


def _lib():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p),
                                                      ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint32)]
        _hip.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
    return _hip


def num_cus(device) -> int:
    return torch.cuda.get_device_properties(device).multi_processor_count


def cu_range(device, spec: str) -> list[int]:
    """'64' -> the last 64 CUs; '-192' -> the first 192; 'a:b' -> CUs a..b-1."""
    n = num_cus(device)
    if ":" in spec:
        a, b = (int(x) for x in spec.split(":"))
    elif spec.startswith("-"):
        a, b = 0, int(spec[1:])
    else:
        a, b = n - int(spec), n
    a, b = max(0, a), min(n, b)
    if a >= b:
        raise ValueError(f"empty CU range {spec!r} on a {n}-CU device")
    return list(range(a, b))


def masked_stream(device, cus: list[int]) -> torch.cuda.ExternalStream:
    """A new stream on ``device`` whose kernels run only on the CUs in ``cus``."""
    n = num_cus(device)
    words = (n + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = _lib().hipExtStreamCreateWithCUMask(ctypes.byref(s), words, mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
    return torch.cuda.ExternalStream(s.value, device=device)
