"""Hand-written persistent MFMA GEMM (ops/csrc/gemm.hip) with fused epilogues.

``gemm_nt(a, b)`` computes ``a @ b.T`` (both operands K-contiguous bf16). The epilogue
variants fold the GPT-2 MLP's elementwise passes into the GEMM that produces them:

* ``epi="bias"``       ``a @ b.T + bias``
* ``epi="bias_gelu"``  returns ``(gelu_tanh(acc + bias), acc)`` — activation and the
  pre-activation saved for backward, one GEMM, no separate bias+GELU pass.
* ``epi="dgelu"``      ``(a @ b.T) * gelu_tanh'(aux + bias)`` plus the bias gradient
  (column sums, accumulated into ``db``) — the MLP's input-gradient GEMM, GELU backward
  and bias reduction in one kernel + one tiny colsum.

Shape contract (checked in C): K % 64 == 0, N % 4 == 0, rows 16-byte aligned.
"""

from __future__ import annotations

import os

import torch

from ._lib import check, lib, ptr, stream_ptr

_EPI = {"none": 0, "bias": 1, "bias_gelu": 2, "dgelu": 3}

# Status: correct (tests/test_kernels_gpu.py::test_gemm_nt_matches_fp32) but measured at
# 0.43-0.77x hipBLASLt on the GPT-2 shapes (profiles/r2/hip_gemm_v*.log), so the model's
# linear layers stay on hipBLASLt; this module is the API for callers that want the fused
# epilogues (scripts/hip_gemm_bench.py). The persistent grid is sized by the kernel.
GRID_CAP = 0


def supported(a: torch.Tensor, b: torch.Tensor) -> bool:
    return (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
            and a.dim() == 2 and b.dim() == 2 and a.shape[1] == b.shape[1]
            and a.shape[1] % 64 == 0 and b.shape[0] % 4 == 0 and a.stride(1) == 1
            and b.stride(1) == 1 and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0)


def gemm_nt(a: torch.Tensor, b: torch.Tensor, *, epi: str = "none", bias=None, aux=None,
            out=None, db=None, db_acc: bool = False):
    """C = epi(a @ b.T). See module docstring for the epilogues."""
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=torch.bfloat16)
    e = _EPI[epi]
    colpart = scratch = None
    flags = 0
    if epi == "bias_gelu" and aux is None:
        aux = torch.empty(M, N, device=a.device, dtype=torch.bfloat16)
    if epi == "dgelu":
        L = lib()
        work = torch.empty(L.ra_gemm_dgelu_work(M, N), device=a.device, dtype=torch.float32)
        P = (M + 127) // 128
        colpart = work[: P * N]
        scratch = work[P * N:]
        if db is not None:
            flags = (1 if db.dtype == torch.bfloat16 else 0) | (2 if db_acc else 0)
    check(lib().ra_gemm_nt(ptr(a), a.stride(0), ptr(b), b.stride(0), ptr(out), out.stride(0), M, N, K, e,
             ptr(bias), ptr(aux), aux.stride(0) if aux is not None else 0, ptr(colpart), ptr(db),
             ptr(scratch), flags, GRID_CAP, stream_ptr()), "gemm_nt")
    if epi == "bias_gelu":
        return out, aux
    return out


def transposed(w: torch.Tensor) -> torch.Tensor:
    """w.T made contiguous: the input-gradient GEMM's B operand (dY @ w = gemm_nt(dY, w.T)).
    Not cached across calls: the flat optimizer updates parameters through raw pointers,
    which torch's version counter does not see. ~2 x |w| bytes of HBM traffic."""
    return w.t().contiguous()
