"""fp32-output bf16 GEMMs on hipBLASLt with per-shape solution selection
(``ops/csrc/gemm_lt.hip``).

``wgrad_accum(dy, x, sink)`` accumulates ``dy^T @ x`` (bf16 operands, fp32 math) straight
into an fp32 gradient buffer: the buffer is the GEMM's C/D operand with beta = 1, so no
split-K partials are written and re-read. Every problem shape uses the fastest of
hipBLASLt's heuristic candidates:

  * choices are read from ``ray_amd/tuned/lt_f32out.csv`` (committed next to the
    TunableOp file for the bf16-output GEMMs);
  * ``RAY_AMD_LT_TUNE=1`` (or ``set_tuning(True)``) times every candidate of a shape on
    its first use (into a scratch buffer) and records the winner; ``save()`` writes the
    file. Without a recorded choice and without tuning, the first heuristic candidate
    runs (hipBLASLt's own pick).
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch

from . import _lib
from ._lib import check, ptr, stream_ptr

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_FILE = os.path.join(os.path.dirname(_HERE), "tuned", "lt_f32out.csv")

_lock = threading.Lock()
_choices: dict | None = None  # key str -> (choice, ms)
_applied: set = set()
_tuning = os.environ.get("RAY_AMD_LT_TUNE", "0") == "1"
_file = os.environ.get("RAY_AMD_LT_FILE", DEFAULT_FILE)


def set_tuning(on: bool, path: str | None = None):
    global _tuning, _file
    _tuning = bool(on)
    if path:
        _file = path


def _load():
    global _choices
    if _choices is not None:
        return _choices
    _choices = {}
    if os.path.exists(_file):
        with open(_file) as f:
            for line in f:
                parts = line.strip().split(",")
                if len(parts) == 3 and parts[0].startswith("lt_"):
                    _choices[parts[0]] = (int(parts[1]), float(parts[2]))
    return _choices


def save(path: str | None = None):
    ch = _load()
    p = path or _file
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        for k in sorted(ch):
            f.write(f"{k},{ch[k][0]},{ch[k][1]:.5f}\n")
    return p


def choice_name(ta, tb, m, n, k, lda, ldb, ldc, batch=1, sa=0, sb=0, sc=0) -> str:
    """Kernel name of the solution a shape currently runs (diagnostics, tests)."""
    buf = ctypes.create_string_buffer(512)
    idx = _lib.lib().ra_lt_choice_name(ta, tb, m, n, k, lda, ldb, ldc, batch, sa, sb, sc, buf,
                                       512)
    if idx < 0:
        raise RuntimeError("hipBLASLt has no solution for this shape")
    return buf.value.decode()


def wgrad_choice_name(M: int, N: int, K: int, S: int = 1) -> str:
    """Kernel of the fp32-out weight-gradient GEMM dy[M, N]^T x[M, K] (S = split-K slices)."""
    if S == 1:
        return choice_name(0, 1, K, N, M, K, N, K)
    Ms = M // S
    return choice_name(0, 1, K, N, Ms, K, N, K, S, Ms * K, Ms * N, N * K)


def is_streamk(name: str) -> bool:
    import re

    return bool(re.search(r"_SK\d", name)) or "StreamK" in name


def _key(ta, tb, m, n, k, lda, ldb, ldc, batch=1, sa=0, sb=0, sc=0):
    base = f"lt_{ta}{tb}_{m}_{n}_{k}_{lda}_{ldb}_{ldc}"
    return base if batch == 1 else f"{base}_b{batch}_{sa}_{sb}_{sc}"


def _select(ta, tb, m, n, k, A, lda, B, ldb, ldc, dev, batch=1, sa=0, sb=0, sc=0):
    shape = (ta, tb, m, n, k, lda, ldb, ldc)
    bshape = (batch, sa, sb, sc)
    key = _key(*shape, *bshape)
    if key in _applied:
        return
    with _lock:
        if key in _applied:
            return
        L = _lib.lib()
        nc = L.ra_lt_num_cands_batched(*shape, *bshape)
        if nc <= 0:
            raise RuntimeError(f"hipBLASLt has no solution for {key}")
        ch = _load()
        # a recorded choice that is a stream-K kernel is refused (rc -2, the plan keeps its
        # first non-stream-K candidate; gemm_lt.hip explains the deadlock it avoids)
        if key in ch and ch[key][0] < nc and \
                L.ra_lt_set_choice_batched(*shape, *bshape, ch[key][0]) == 0:
            pass
        elif _tuning:
            scratch = torch.empty(ldc * n + sc * (batch - 1), dtype=torch.float32, device=dev)
            best = ctypes.c_float(0.0)
            idx = L.ra_lt_tune(ta, tb, m, n, k, A, lda, B, ldb, ptr(scratch), ldc, 5,
                               ctypes.addressof(best), batch, sa, sb, sc, stream_ptr())
            if idx >= 0:
                ch[key] = (idx, best.value)
            del scratch
        _applied.add(key)


def gemm_f32(ta: int, tb: int, m: int, n: int, k: int, A, lda: int, B, ldb: int, C, ldc: int,
             alpha: float = 1.0, beta: float = 0.0, batch: int = 1, sa: int = 0, sb: int = 0,
             sc: int = 0):
    """Column-major C[m x n] (fp32) = alpha * op(A) * op(B) + beta * C, bf16 A/B; with
    batch > 1 the operands of GEMM i start at base + i * stride (elements)."""
    _select(ta, tb, m, n, k, ptr(A), lda, ptr(B), ldb, ldc, C.device, batch, sa, sb, sc)
    if batch == 1:
        rc = _lib.lib().ra_lt_gemm(ta, tb, m, n, k, ptr(A), lda, ptr(B), ldb, ptr(C), ldc,
                                   float(alpha), float(beta), stream_ptr())
    else:
        rc = _lib.lib().ra_lt_gemm_batched(ta, tb, m, n, k, ptr(A), lda, sa, ptr(B), ldb, sb,
                                           ptr(C), ldc, sc, batch, float(alpha), float(beta),
                                           stream_ptr())
    check(rc, "lt_gemm")


def wgrad_partials(dy2: torch.Tensor, x2: torch.Tensor, S: int) -> torch.Tensor:
    """Split-K weight gradient: part[s] (fp32 [N, K]) = dy2_s^T @ x2_s over S token slices,
    one tuned strided-batched GEMM (summed afterwards by ra_splitk_accum)."""
    M, N = dy2.shape
    K = x2.shape[1]
    Ms = M // S
    part = torch.empty((S, N, K), dtype=torch.float32, device=dy2.device)
    gemm_f32(0, 1, K, N, Ms, x2, K, dy2, N, part, K, batch=S, sa=Ms * K, sb=Ms * N, sc=N * K)
    return part


def wgrad_accum(dy2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor, beta: float = 1.0,
                alpha: float = 1.0):
    """out[N, K] (fp32, row-major) = alpha * dy2[M, N]^T @ x2[M, K] + beta * out.

    Row-major out[N, K] is column-major out^T[K x N]: out^T = x2^T * dy2 with x2 read as a
    column-major [K x M] matrix (no transpose) and dy2 as [N x M] transposed."""
    M, N = dy2.shape
    K = x2.shape[1]
    assert x2.shape[0] == M and out.shape == (N, K) and out.dtype == torch.float32
    assert dy2.stride(1) == 1 and x2.stride(1) == 1 and out.is_contiguous()
    gemm_f32(0, 1, K, N, M, x2, x2.stride(0), dy2, dy2.stride(0), out, K, alpha, beta)


def release_stream(stream) -> int:
    """Free the hipBLASLt handle and workspace cached for ``stream`` (ra_lt_release_stream).
    Owners of short-lived streams call it once no more lt GEMMs run there and no captured
    graph refers to the stream's workspace. torch hands out streams from a fixed per-device
    pool, so the cached set is bounded even without it; a release returns the 64 MiB
    workspaces early. Returns the number of entries freed (0 when the stream never ran an
    lt GEMM)."""
    from ._lib import lib

    return int(lib().ra_lt_release_stream(stream.cuda_stream))
