"""Autograd-aware entry points for the CDNA4 kernels.

Every op dispatches on device: CUDA(HIP) tensors go to the hand-written kernels
in ``libray_amd_hip.so`` (failing loudly if it is missing), CPU tensors go to the
fp32 references in ``ray_amd.ops.reference``.
"""

from __future__ import annotations

import os

import torch

from . import _lib
from . import reference as ref
from ._lib import check, ptr, stream_ptr


def _hip(t: torch.Tensor) -> bool:
    return t.is_cuda


# --------------------------------------------------------------------- flat-grad sinks
# Parameters managed by ray_amd.parallel.flat carry ``_ra_grad``: a view into ONE flat
# gradient buffer (fp32 by default, bf16 when gradient compression is on), and are
# tagged ``_ra_direct_grad``. Our backward kernels then ACCUMULATE their parameter
# gradients straight into that view (fp32 math, one HBM pass) and return None, so
# autograd never allocates a gradient tensor nor launches an AccumulateGrad add; the
# DDP bucket hook (``_ra_grad_ready``) is signalled exactly once per backward instead.
def _grad_sink(p):
    if p is not None and getattr(p, "_ra_direct_grad", False):
        return getattr(p, "_ra_grad", None)
    return None


def _sink_f32(t) -> int:
    return 1 if t is not None and t.dtype == torch.float32 else 0


def _grad_done(p):
    cb = getattr(p, "_ra_grad_ready", None)
    if cb is not None:
        cb()


# --------------------------------------------------------------------- LayerNorm
def _ln_forward(x, w, b, eps):
    D = x.shape[-1]
    x2 = x.contiguous().view(-1, D)
    N = x2.shape[0]
    y = torch.empty_like(x2)
    mean = torch.empty(N, device=x.device, dtype=torch.float32)
    rstd = torch.empty(N, device=x.device, dtype=torch.float32)
    check(_lib.lib().ra_layernorm_fwd(ptr(x2), ptr(w), ptr(b), ptr(y), ptr(mean), ptr(rstd),
                                      N, D, eps, stream_ptr()), "layernorm_fwd")
    return x2, y, mean, rstd


def _ln_backward(dy, x2, w, b, mean, rstd, dres=None, rbias=None):
    """dx (+ dres) and the weight/bias grads (into flat sinks when available). With
    ``rbias`` (the bias of the residual add that produced x) also its gradient colsum(dx).
    Returns (dx, dw, db, drbias) with None for gradients accumulated in place."""
    N, D = x2.shape
    dy2 = dy.contiguous().view(N, D)
    L = _lib.lib()
    work = torch.empty(L.ra_layernorm_bwd_work(N, D), device=dy.device, dtype=torch.float32)
    dx = torch.empty_like(x2)
    params = [w, b] + ([rbias] if rbias is not None else [])
    sinks = [_grad_sink(p) for p in params]
    direct = all(s_ is not None for s_ in sinks)
    outs = sinks if direct else [torch.empty_like(p) for p in params]
    if rbias is None:
        outs.append(None)
    flags = (1 if outs[0].dtype == torch.bfloat16 else 0) | (2 if direct else 0)
    dr = None if dres is None else dres.contiguous().view(N, D)
    check(L.ra_layernorm_bwd(ptr(dy2), ptr(x2), ptr(w), ptr(mean), ptr(rstd), ptr(dr), ptr(dx),
                             ptr(outs[0]), ptr(outs[1]), ptr(outs[2]), ptr(work), N, D, flags,
                             stream_ptr()), "layernorm_bwd")
    if direct:
        for p in params:
            _grad_done(p)
        return dx, None, None, None
    return dx, outs[0], outs[1], outs[2]


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        x2, y, mean, rstd = _ln_forward(x, w, b, eps)
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.b = b
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dx, dw, db, _ = _ln_backward(dy, x2, w, ctx.b, mean, rstd)
        return dx.view(ctx.shape), dw, db, None


class _LayerNormFork(torch.autograd.Function):
    """(x, LN(x)) for a pre-LN residual block: the residual stream's two gradients (through
    the skip connection and through LN) are summed inside the LN backward kernel."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        x2, y, mean, rstd = _ln_forward(x, w, b, eps)
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.b = b
        ctx.shape = x.shape
        return x.view_as(x), y.view(x.shape)

    @staticmethod
    def backward(ctx, dskip, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dx, dw, db, _ = _ln_backward(dy, x2, w, ctx.b, mean, rstd, dres=dskip)
        return dx.view(ctx.shape), dw, db, None


class _ResidualLayerNorm(torch.autograd.Function):
    """x = h + rbias + skip ; (x, LN(x)) in one kernel. Backward: one kernel computes
    dx = dskip_out + LN_bwd(dy) and the column sums for dgamma, dbeta AND d(rbias)."""

    @staticmethod
    def forward(ctx, h, rbias, skip, w, b, eps):
        D = h.shape[-1]
        h2 = h.contiguous().view(-1, D)
        s2 = skip.contiguous().view(-1, D)
        N = h2.shape[0]
        xo = torch.empty_like(h2)
        y = torch.empty_like(h2)
        mean = torch.empty(N, device=h.device, dtype=torch.float32)
        rstd = torch.empty(N, device=h.device, dtype=torch.float32)
        check(_lib.lib().ra_residual_layernorm_fwd(ptr(h2), ptr(rbias), ptr(s2), ptr(xo), ptr(w),
                                                   ptr(b), ptr(y), ptr(mean), ptr(rstd), N, D,
                                                   eps, stream_ptr()), "residual_layernorm_fwd")
        ctx.save_for_backward(xo, w, mean, rstd)
        ctx.b, ctx.rbias = b, rbias
        ctx.shape = h.shape
        return xo.view(h.shape), y.view(h.shape)

    @staticmethod
    def backward(ctx, dxo, dy):
        xo, w, mean, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(xo)
        dx, dw, db, drb = _ln_backward(dy, xo, w, ctx.b, mean, rstd, dres=dxo,
                                       rbias=ctx.rbias)
        dx = dx.view(ctx.shape)
        return dx, drb, dx, dw, db, None


def residual_layer_norm(h, rbias, skip, weight, bias, eps=1e-5):
    """Pre-LN transformer seam: x = h + rbias + skip; returns (x, LayerNorm(x))."""
    if _hip(h) and h.dtype == torch.bfloat16 and h.shape[-1] % 8 == 0 and rbias is not None:
        return _ResidualLayerNorm.apply(h, rbias, skip, weight, bias, eps)
    x = ref.bias_residual(h, rbias, skip) if rbias is not None else h + skip
    return x, ref.layer_norm(x, weight, bias, eps)


def layer_norm(x, weight, bias, eps=1e-5):
    if _hip(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 4 == 0:
        return _LayerNorm.apply(x, weight, bias, eps)
    return ref.layer_norm(x, weight, bias, eps)


def layer_norm_fork(x, weight, bias, eps=1e-5):
    """Returns (x_skip, layer_norm(x)); use x_skip for the residual add."""
    if _hip(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 4 == 0:
        return _LayerNormFork.apply(x, weight, bias, eps)
    return x, ref.layer_norm(x, weight, bias, eps)


# --------------------------------------------------------------------- bias + GELU
class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, bias):
        F_ = h.shape[-1]
        h2 = h.contiguous().view(-1, F_)
        y = torch.empty_like(h2)
        check(_lib.lib().ra_bias_gelu_fwd(ptr(h2), ptr(bias), ptr(y), h2.shape[0], F_,
                                          stream_ptr()), "bias_gelu_fwd")
        ctx.save_for_backward(h2)
        ctx.bias = bias
        ctx.shape = h.shape
        return y.view(h.shape)

    @staticmethod
    def backward(ctx, dy):
        (h2,) = ctx.saved_tensors
        bias = ctx.bias
        N, F_ = h2.shape
        L = _lib.lib()
        work = torch.empty(L.ra_colsum_work(N, F_), device=dy.device, dtype=torch.float32)
        dh = torch.empty_like(h2)
        sink = _grad_sink(bias)
        db = sink if sink is not None else torch.empty_like(bias)
        flags = (1 if sink is not None else 0) | (2 * _sink_f32(db))
        check(L.ra_bias_gelu_bwd(ptr(dy.contiguous()), ptr(h2), ptr(bias), ptr(dh), ptr(db),
                                 ptr(work), N, F_, flags, stream_ptr()), "bias_gelu_bwd")
        if sink is not None:
            _grad_done(bias)
            return dh.view(ctx.shape), None
        return dh.view(ctx.shape), db


def bias_gelu(h, bias):
    if _hip(h) and h.dtype == torch.bfloat16 and h.shape[-1] % 8 == 0:
        return _BiasGelu.apply(h, bias)
    return ref.bias_gelu(h, bias)


# --------------------------------------------------------------------- bias + residual
def _colsum_bf16(x2, out=None):
    """Column sum of [N, F] bf16 -> [F] bf16; with `out` given (bf16 or fp32), accumulate
    into it."""
    N, F_ = x2.shape
    L = _lib.lib()
    work = torch.empty(L.ra_colsum_work(N, F_), device=x2.device, dtype=torch.float32)
    acc = out is not None
    if out is None:
        out = torch.empty(F_, device=x2.device, dtype=x2.dtype)
    check(L.ra_colsum_bf16(ptr(x2), ptr(out), ptr(work), N, F_,
                           (1 if acc else 0) | 2 * _sink_f32(out), stream_ptr()), "colsum")
    return out


def _bias_grad(dy2, bias):
    """bias gradient: accumulated into the flat sink (returns None) or a new tensor."""
    sink = _grad_sink(bias)
    if sink is not None:
        _colsum_bf16(dy2, out=sink)
        _grad_done(bias)
        return None
    return _colsum_bf16(dy2)


class _BiasResidual(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, bias, res):
        F_ = h.shape[-1]
        h2 = h.contiguous().view(-1, F_)
        r2 = res.contiguous().view(-1, F_)
        y = torch.empty_like(h2)
        check(_lib.lib().ra_bias_residual(ptr(h2), ptr(bias), ptr(r2), ptr(y), h2.shape[0], F_,
                                          stream_ptr()), "bias_residual")
        ctx.bias = bias
        return y.view(h.shape)

    @staticmethod
    def backward(ctx, dy):
        db = None
        if ctx.bias is not None and ctx.needs_input_grad[1]:
            db = _bias_grad(dy.contiguous().view(-1, dy.shape[-1]), ctx.bias)
        return dy, db, dy


def bias_residual(h, bias, res):
    if _hip(h) and h.dtype == torch.bfloat16 and h.shape[-1] % 8 == 0:
        return _BiasResidual.apply(h, bias, res)
    return ref.bias_residual(h, bias, res)


# --------------------------------------------------------------------- linear (split-K wgrad)
# Weight gradients (fp32 out) run the hand-written CDNA4 kernel (ops/csrc/wgrad.hip, bias
# gradient fused; measured -2.3 ms/step vs hipBLASLt split-K partials on MI355X,
# profiles/r5/r5c). Layouts that kernel does not take fall back to fp32 split-K partials
# from S token-slice GEMMs (torch.bmm on the main stream, ops/lt's per-stream hipBLASLt
# handle on the side stream) summed into the sink by one HIP pass.
# RAY_AMD_WGRAD_STREAM=1 (default): weight gradients run on a side stream
_WGRAD_STREAM = os.environ.get("RAY_AMD_WGRAD_STREAM", "1") == "1"

# fallback split-K: at most 16 token slices of >= 2048 tokens, <= 4 GiB of fp32 partials
# (profiles/r2_perf_bench.log: S = 16 fastest for every GPT-2 projection on hipBLASLt)
_WGRAD_MAX_SPLITS = 16
_WGRAD_PART_BYTES = 4 << 30


def _splitk(M: int, N: int, K: int) -> int:
    """Token slices for the fallback split-K weight gradient."""
    S = 1
    while (S < _WGRAD_MAX_SPLITS and M % (2 * S) == 0 and M // (2 * S) >= 2048
           and 2 * S * N * K * 4 <= _WGRAD_PART_BYTES):
        S *= 2
    return S


def _on_side_stream(t) -> bool:
    st = _side.get(t.device)
    return st is not None and torch.cuda.current_stream(t.device) == st


def _wgrad_partials(dy2, x2, S, M, N, K):
    """fp32 split-K partials [S, N, K]. On the wgrad side stream they always come from
    ops/lt (a per-stream hipBLASLt handle): torch.bmm would share torch's one handle with
    the main stream's dX GEMM, the concurrent stream-K setup that hung in round 4."""
    side = dy2.is_cuda and _on_side_stream(dy2)
    if side:
        from . import lt

        return lt.wgrad_partials(dy2.contiguous(), x2.contiguous(), S)
    return torch.bmm(dy2.view(S, M // S, N).transpose(1, 2), x2.view(S, M // S, K),
                     out_dtype=torch.float32)


def _wgrad_hip_ok(dy2, x2, sink, bias_sink=None) -> bool:
    M, N = dy2.shape
    K = x2.shape[1]
    return (dy2.is_cuda and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16
            and M >= 64 and N % 8 == 0 and K % 8 == 0
            and dy2.stride(1) == 1 and x2.stride(1) == 1
            and dy2.stride(0) % 8 == 0 and x2.stride(0) % 8 == 0
            and dy2.data_ptr() % 16 == 0 and x2.data_ptr() % 16 == 0
            and sink.is_contiguous() and sink.numel() == N * K
            and sink.dtype in (torch.float32, torch.bfloat16) and sink.data_ptr() % 16 == 0
            and (bias_sink is None or (bias_sink.dtype == sink.dtype
                                       and bias_sink.is_contiguous()
                                       and bias_sink.numel() == N)))


def wgrad_accumulate(dy2, x2, sink, bias_sink=None, accumulate=True):
    """sink[N, K] (+)= dy2[M, N]^T @ x2[M, K] and, with ``bias_sink``, bias_sink[N] (+)=
    colsum(dy2) — the hand-written CDNA4 weight-gradient kernel (ops/csrc/wgrad.hip: both
    operands read token-major through LDS transpose reads, split-K over tokens sized to one
    wave of workgroups, fp32 slabs summed into the sink by one pass). ``sink``/``bias_sink``
    are fp32 or bf16 (same dtype); fp32 math throughout. A token tail (M % 64) is added by
    an fp32 torch GEMM. Use ``_wgrad_hip_ok`` to check the layout first."""
    M, N = dy2.shape
    K = x2.shape[1]
    L = _lib.lib()
    Mk = M - M % 64
    flags = (1 if sink.dtype == torch.bfloat16 else 0) | (2 if accumulate else 0) | \
        (4 if bias_sink is not None else 0)
    S = L.ra_wgrad_splits(Mk, N, K)
    if S == 1:
        check(L.ra_wgrad(ptr(dy2), dy2.stride(0), ptr(x2), x2.stride(0), Mk, N, K, 1, ptr(sink),
                         ptr(bias_sink), flags, stream_ptr()), "wgrad")
    else:
        ws = torch.empty(S * N * K + (S * N if bias_sink is not None else 0),
                         device=dy2.device, dtype=torch.float32)
        bws = ws[S * N * K:] if bias_sink is not None else None
        check(L.ra_wgrad(ptr(dy2), dy2.stride(0), ptr(x2), x2.stride(0), Mk, N, K, S, ptr(ws),
                         ptr(bws), flags, stream_ptr()), "wgrad")
        acc = (1 if accumulate else 0) | 2 * _sink_f32(sink)
        check(L.ra_splitk_accum(ptr(ws), S, N * K, ptr(sink), acc, stream_ptr()), "splitk_accum")
        if bias_sink is not None:
            check(L.ra_splitk_accum(ptr(bws), S, N, ptr(bias_sink), acc, stream_ptr()),
                  "splitk_accum")
    if Mk < M:  # token tail: an fp32 GEMM on at most 63 rows
        dt, xt = dy2[Mk:].float(), x2[Mk:].float()
        sv = sink.view(N, K)
        sv.copy_(sv.float().addmm_(dt.t(), xt))
        if bias_sink is not None:
            bias_sink.copy_(bias_sink.float() + dt.sum(0))


def _wgrad_to_sink(dy2, x2, w, sink, S, M, N, K, bias=None, bias_sink=None):
    """sink += dy2^T x2 (fp32 or bf16 flat-gradient view), then signal DDP readiness. With
    ``bias_sink`` (hip path only) the bias gradient is fused into the same kernel."""
    if _wgrad_hip_ok(dy2, x2, sink, bias_sink):
        wgrad_accumulate(dy2, x2, sink, bias_sink)
        _grad_done(w)
        if bias_sink is not None:
            _grad_done(bias)
        return
    if bias_sink is not None:  # layout not supported by the fused kernel: separate colsum
        _colsum_bf16(dy2, out=bias_sink)
        _grad_done(bias)
    # fp32 partials [S, N, K] from S token-slice GEMMs, summed (+ accumulated into the flat
    # gradient) by one HIP pass
    part = _wgrad_partials(dy2, x2, S, M, N, K)
    check(_lib.lib().ra_splitk_accum(ptr(part), S, N * K, ptr(sink),
                                     1 | 2 * _sink_f32(sink), stream_ptr()), "splitk_accum")
    _grad_done(w)


_side: dict = {}

def _issue_side_wgrad(job):
    dy2, x2, w, sink, S, M, N, K, b, bsink = job
    side = _side_stream(dy2.device)
    side.wait_stream(torch.cuda.current_stream(dy2.device))
    with torch.cuda.stream(side):
        _wgrad_to_sink(dy2, x2, w, sink, S, M, N, K, b, bsink)
        dy2.record_stream(side)
        x2.record_stream(side)


def _side_stream(device):
    st = _side.get(device)
    if st is None:
        st = _side[device] = torch.cuda.Stream(device)
    return st


def join_side_streams():
    """Make the current stream wait for weight-gradient work queued on side streams (call
    before consuming the flat gradients: optimizer step, collective)."""
    for dev, st in _side.items():
        torch.cuda.current_stream(dev).wait_stream(st)


# Host run-ahead bound for steps that use the side stream. A block that another stream used
# (record_stream) returns to the caching allocator only once an event recorded at its free
# has completed. The host enqueues a step in less time than the GPU runs it, so with no bound
# every step's activations and logits were still pending when the next steps allocated, and
# the cache grew by ~7 GB per step: r5ac measured 1011 hipMallocs and 284 GB reserved against
# 27.7 GB allocated (the single-stream step: 131 and 28 GB). The next process on the GPU then
# waits out the teardown of that reservation (profiles/r5/r5p). bound_run_ahead() is called
# once per optimizer step: the host waits until the GPU reached the same point
# RAY_AMD_RUN_AHEAD steps earlier, which still leaves a whole step queued (0 = unbounded).
_RUN_AHEAD = int(os.environ.get("RAY_AMD_RUN_AHEAD", "1"))
_step_marks: dict = {}


def bound_run_ahead():
    if _RUN_AHEAD <= 0 or not _side or torch.cuda.is_current_stream_capturing():
        return
    import collections

    dev = torch.cuda.current_device()
    q = _step_marks.get(dev)
    if q is None:
        q = _step_marks[dev] = collections.deque()
    ev = torch.cuda.Event()
    ev.record()
    q.append(ev)
    while len(q) > _RUN_AHEAD:
        q.popleft().synchronize()


# RAY_AMD_DGRAD_WT (default on; 0 disables): the input-gradient GEMM dX = dY @ W reads a transposed bf16 copy of
# W ([in, out], refreshed once per optimizer step on the side stream during the forward),
# so it runs in the forward GEMMs' operand layout (TunableOp "tn" instead of "nn";
# scripts/dgrad_layout_ab.py measures both). Costs one extra bf16 copy of every weight.
# Measured on MI355X (profiles/r4/r4g): 67.09 vs 67.59 ms/step, three interleaved pairs.
_DGRAD_WT = os.environ.get("RAY_AMD_DGRAD_WT", "1") == "1"
_weights_epoch = [0]


def bump_weights_epoch():
    """Called after every in-place weight update that bypasses autograd's version counter
    (the flat AdamW kernel): transposed weight copies are refreshed on next use."""
    _weights_epoch[0] += 1


def weights_epoch() -> int:
    return _weights_epoch[0]


def _transposed_weight(w):
    """(Wt, event): W^T contiguous, refreshed on the side stream when the weights changed
    since the last refresh (always under graph capture, where host state is frozen).

    Weights of a FlatParams built with ``transpose=`` own a W^T view (``_ra_wt_view``) that
    the fused AdamW kernel rewrites every step: it is used as is (no kernel, no event) while
    its validity key matches, and under graph capture (the captured optimizer step keeps it
    fresh on every replay). Any other in-place change of W (copy_, load) bumps its version,
    and the copy is refreshed into the same view by the side-stream transpose."""
    view = getattr(w, "_ra_wt_view", None)
    if view is not None:
        if torch.cuda.is_current_stream_capturing() or \
                getattr(w, "_ra_wt_key", None) == (_weights_epoch[0], w._version):
            return view, getattr(w, "_ra_wt_ev", None)
        side = _side_stream(w.device)
        side.wait_stream(torch.cuda.current_stream(w.device))
        with torch.cuda.stream(side):
            check(_lib.lib().ra_transpose_bf16(ptr(w), ptr(view), w.shape[0], w.shape[1],
                                               side.cuda_stream), "transpose_bf16")
            ev = torch.cuda.Event()
            ev.record(side)
        w._ra_wt_key = (_weights_epoch[0], w._version)
        # later users on the main stream must see the refresh: keep the event until the
        # next optimizer step marks the view fresh again
        w._ra_wt_ev = ev
        return view, ev
    cache = getattr(w, "_ra_wt", None)
    key = (_weights_epoch[0], w._version, w.data_ptr())  # kernel updates, copy_(), rebinding
    stale = cache is None or cache[1] != key or torch.cuda.is_current_stream_capturing()
    if not stale:
        return cache[0], cache[2]
    wt = cache[0] if cache is not None else torch.empty(w.shape[1], w.shape[0], dtype=w.dtype,
                                                        device=w.device)
    side = _side_stream(w.device)
    side.wait_stream(torch.cuda.current_stream(w.device))
    with torch.cuda.stream(side):
        if w.dtype == torch.bfloat16 and w.dim() == 2 and w.is_contiguous():
            check(_lib.lib().ra_transpose_bf16(ptr(w), ptr(wt), w.shape[0], w.shape[1],
                                               side.cuda_stream), "transpose_bf16")
        else:
            wt.copy_(w.detach().t())
        ev = torch.cuda.Event()
        ev.record(side)
    w._ra_wt = (wt, key, ev)
    return wt, ev


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.b = b
        ctx.wt = _transposed_weight(w) if _DGRAD_WT and w.is_cuda and x.dim() >= 2 else None
        return torch.nn.functional.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        K, N = x.shape[-1], w.shape[0]
        x2 = x.reshape(-1, K)
        dy2 = dy.reshape(-1, N)
        M = x2.shape[0]
        dx = None
        if ctx.needs_input_grad[0]:
            if ctx.wt is not None:
                wt, ev = ctx.wt
                if ev is not None:
                    torch.cuda.current_stream(dy2.device).wait_event(ev)
                dx = (dy2 @ wt.t()).view(x.shape)
            else:
                dx = (dy2 @ w).view(x.shape)
        dw = db = None
        # hip wgrad: the bias gradient (colsum of dY) is fused into the weight-gradient kernel
        # when both parameters write flat-gradient sinks of one dtype
        bsink = None
        if ctx.b is not None and ctx.needs_input_grad[2] and ctx.needs_input_grad[1]:
            bsink = _grad_sink(ctx.b)
            ws_ = _grad_sink(w)
            if bsink is not None and (ws_ is None or ws_.dtype != bsink.dtype):
                bsink = None
        if ctx.needs_input_grad[1]:
            sink = _grad_sink(w)
            S = _splitk(M, N, K)
            if sink is not None and _WGRAD_STREAM and dy2.is_cuda:
                # weight gradient on the side stream: it overlaps the memory-bound kernels
                # of the dX chain that continues on the main stream
                _issue_side_wgrad((dy2, x2, w, sink, S, M, N, K, ctx.b, bsink))
            elif sink is not None:
                _wgrad_to_sink(dy2, x2, w, sink, S, M, N, K, ctx.b, bsink)
            elif S > 1:
                part = _wgrad_partials(dy2, x2, S, M, N, K)
                dw = torch.empty_like(w)
                check(_lib.lib().ra_splitk_accum(ptr(part), S, N * K, ptr(dw), 2 * _sink_f32(dw),
                                                 stream_ptr()), "splitk_accum")
            else:
                dw = dy2.t() @ x2
        if ctx.b is not None and ctx.needs_input_grad[2] and bsink is None:
            db = _bias_grad(dy2, ctx.b)
        return dx, dw, db


def linear(x, w, b=None):
    """y = x @ w^T + b with the MI355X backward (split-K fp32 wgrad, in-place flat-grad
    accumulation). Same numerics contract as F.linear."""
    if _hip(x) and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and \
            (w.shape[0] * w.shape[1]) % 4 == 0:
        return _Linear.apply(x, w, b)
    return torch.nn.functional.linear(x, w, b)


# --------------------------------------------------------------------- flash attention
class _FlashAttnQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, scale):
        B, T, _, H, D = qkv.shape
        qkv = qkv.contiguous()
        out = torch.empty((B, T, H, D), device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty((B, H, T), device=qkv.device, dtype=torch.float32)
        check(_lib.lib().ra_attn_fwd(ptr(qkv), ptr(out), ptr(lse), B, T, H, D, scale,
                                     stream_ptr()), "attn_fwd")
        ctx.save_for_backward(qkv, out, lse)
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        B, T, _, H, D = qkv.shape
        dout = dout.contiguous()
        dqkv = torch.empty_like(qkv)
        delta = torch.empty((B, H, T), device=qkv.device, dtype=torch.float32)
        # dQ (with delta = rowsum(dO*O) inside) then dK/dV: no float atomics, bitwise
        # reproducible (measured against a fused one-pass form with fp32 dQ atomics and a
        # two-stream split: profiles/r2/attn_bwd_fused_vs_split.md, profiles/r5/r5au)
        check(_lib.lib().ra_attn_bwd(ptr(qkv), ptr(out), ptr(dout), ptr(lse), ptr(delta),
                                     ptr(dqkv), B, T, H, D, ctx.scale, stream_ptr()),
              "attn_bwd")
        return dqkv, None


def causal_attention_qkv(qkv, scale=None):
    """Causal self-attention from a packed [B, T, 3, H, D] QKV tensor → [B, T, H, D].

    HIP MFMA flash attention for D == 64, T % 128 == 0 (bf16); otherwise PyTorch SDPA."""
    B, T, _, H, D = qkv.shape
    if scale is None:
        scale = D ** -0.5
    if _hip(qkv) and qkv.dtype == torch.bfloat16 and D == 64 and T % 128 == 0:
        return _FlashAttnQKV.apply(qkv, float(scale))
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
    y = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True, scale=scale)
    return y.transpose(1, 2)


# --------------------------------------------------------------------- cross entropy
class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, V, ignore_index):
        Vp = logits.shape[-1]
        l2 = logits.contiguous().view(-1, Vp)
        t = targets.contiguous().view(-1).long()
        N = l2.shape[0]
        loss = torch.empty(N, device=logits.device, dtype=torch.float32)
        lse = torch.empty(N, device=logits.device, dtype=torch.float32)
        check(_lib.lib().ra_xent_fwd(ptr(l2), ptr(t), ptr(loss), ptr(lse), N, V, Vp,
                                     ignore_index, stream_ptr()), "xent_fwd")
        count = (t != ignore_index).sum().clamp_min(1)
        ctx.save_for_backward(l2, t, lse, count)
        ctx.V, ctx.ignore_index, ctx.shape = V, ignore_index, logits.shape
        return loss.sum() / count

    @staticmethod
    def backward(ctx, g):
        l2, t, lse, count = ctx.saved_tensors
        N, Vp = l2.shape
        # fold 1/count into the device-side grad scalar: no host sync
        gs = (g.float() / count.float()).reshape(1).contiguous()
        dl = torch.empty_like(l2)
        check(_lib.lib().ra_xent_bwd(ptr(l2), ptr(t), ptr(lse), ptr(gs), 1.0, ptr(dl), N, ctx.V,
                                     Vp, ctx.ignore_index, stream_ptr()), "xent_bwd")
        return dl.view(ctx.shape), None, None, None


# LM-head weight gradient: the wgrad kernel (split count from ra_wgrad_splits: 3 at 591
# tiles); layouts it does not take use an fp32-out hipBLASLt GEMM — ops/lt (a per-stream
# handle) on the side stream, torch.addmm on the main stream. Two streams issuing stream-K
# hipBLASLt GEMMs through ONE handle hung the GPU in round 4 (profiles/r4/README.md §2).
# With a flat-gradient sink, dW runs once over all tokens on the wgrad side stream, overlapping
# the transformer backward (measured equal to or faster than the main stream, r5g / r5am);
# its scaled accumulation into the sink stays there and the embedding's backward (the
# other user of the tied weight's sink) waits on its event.
def _lm_head_dw(lg, h2s, dw, first, side=False):
    if _wgrad_hip_ok(lg, h2s, dw):
        wgrad_accumulate(lg, h2s, dw, accumulate=not first)
        return
    if side:
        from . import lt

        lt.wgrad_accum(lg, h2s, dw, beta=0.0 if first else 1.0)
    else:
        torch.addmm(dw, lg.t(), h2s, out_dtype=torch.float32, beta=0.0 if first else 1.0,
                    out=dw)


class _LMHeadCrossEntropy(torch.autograd.Function):
    """Tied LM head + mean token cross-entropy, chunked over tokens so the full
    [tokens, vocab] logits never exist. Forward computes the loss AND the gradients
    (the standard fused-linear-cross-entropy trick): per chunk one hipBLASLt GEMM for the
    logits, ``ra_xent_fused`` turning them into dlogits in place, and two GEMMs for dh
    and dW (fp32 accumulate). Backward only scales by the upstream gradient and
    accumulates dW into the flat fp32 (or bf16) gradient sink.

    ``signal_w=False`` for a tied weight whose other use (the embedding) runs later in
    backward and signals DDP readiness itself."""

    @staticmethod
    def forward(ctx, h, w, targets, V, ignore_index, chunk, signal_w):
        C = h.shape[-1]
        h2 = h.contiguous().view(-1, C)
        t = targets.contiguous().view(-1).long()
        N, Vp = h2.shape[0], w.shape[0]
        dev = h.device
        count = (t != ignore_index).sum().clamp_min(1).float()
        inv = (1.0 / count).reshape(1)
        loss_rows = torch.empty(N, device=dev, dtype=torch.float32)
        need_grad = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        dh = torch.empty_like(h2) if need_grad else None
        dw = torch.zeros(w.shape, device=dev, dtype=torch.float32) \
            if ctx.needs_input_grad[1] else None
        ch = max(1, min(chunk, N))
        L = _lib.lib()
        wt = w.t()
        # Token chunks in order on this stream: logits GEMM -> in-place cross-entropy ->
        # dh GEMM, each chunk's logits small enough to stay in the Infinity Cache between
        # the three passes when chunk is small. With a flat-gradient sink the dlogits of
        # all chunks are kept ([N, Vp]) and dW runs ONCE over all tokens on the wgrad side
        # stream (no per-chunk read-modify-write of the fp32 dW); otherwise dW accumulates
        # per chunk on this stream into a chunk-sized logits buffer.
        side_dw = (dw is not None and h.is_cuda and _WGRAD_STREAM
                   and _grad_sink(w) is not None)
        lg = torch.empty((N if side_dw else ch, Vp), device=dev, dtype=h.dtype)
        for s0 in range(0, N, ch):
            e = min(N, s0 + ch)
            lgc = lg[s0:e] if side_dw else lg[: e - s0]
            torch.mm(h2[s0:e], wt, out=lgc)
            check(L.ra_xent_fused(ptr(lgc), ptr(t[s0:e]), ptr(inv), ptr(loss_rows[s0:e]),
                                  e - s0, V, Vp, ignore_index, stream_ptr()), "xent_fused")
            if dh is not None:
                torch.mm(lgc, w, out=dh[s0:e])
            if dw is not None and not side_dw:
                _lm_head_dw(lgc, h2[s0:e], dw, s0 == 0)
        if side_dw:
            side = _side_stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                _lm_head_dw(lg, h2, dw, True, side=True)
            for t_ in (lg, h2, dw):
                t_.record_stream(side)
        ctx.side_dw = side_dw
        ctx.save_for_backward(dh, dw)
        ctx.w, ctx.shape, ctx.signal_w = w, h.shape, signal_w
        return loss_rows.sum() * inv[0]

    @staticmethod
    def backward(ctx, g):
        dh, dw = ctx.saved_tensors
        L = _lib.lib()
        gs = g.float().reshape(1).contiguous()
        dhv = None
        if dh is not None and ctx.needs_input_grad[0]:
            check(L.ra_scale_bf16(ptr(dh), dh.numel(), ptr(gs), stream_ptr()), "scale_bf16")
            dhv = dh.view(ctx.shape)
        dwv = None
        if dw is not None:
            sink = _grad_sink(ctx.w)
            if sink is not None and ctx.side_dw:
                # dW was computed on the side stream: scale + accumulate there too, and
                # leave an event for the other writer of this sink (the embedding)
                side = _side_stream(dw.device)
                side.wait_stream(torch.cuda.current_stream(dw.device))
                with torch.cuda.stream(side):
                    check(L.ra_scaled_accum(ptr(dw), ptr(sink), dw.numel(), _sink_f32(sink),
                                            ptr(gs), stream_ptr()), "scaled_accum")
                    gs.record_stream(side)
                    ev = torch.cuda.Event()
                    ev.record(side)
                    ctx.w._ra_sink_event = ev
                    if ctx.signal_w:
                        _grad_done(ctx.w)
            elif sink is not None:
                check(L.ra_scaled_accum(ptr(dw), ptr(sink), dw.numel(), _sink_f32(sink), ptr(gs),
                                        stream_ptr()), "scaled_accum")
                if ctx.signal_w:
                    _grad_done(ctx.w)
            else:
                dwv = (dw * gs).to(ctx.w.dtype)
        return dhv, dwv, None, None, None, None, None


def lm_head_cross_entropy(h, w, targets, vocab_size=None, ignore_index=-100, chunk=8192,
                          signal_w=True):
    """mean CE(h @ w^T, targets) with w [padded_vocab, C]; columns >= vocab_size are
    excluded from the softmax. HIP path never materialises the full logits."""
    V = vocab_size or w.shape[0]
    if _hip(h) and h.dtype == torch.bfloat16 and w.shape[0] % 8 == 0 and \
            (w.shape[0] // 8 + 511) // 512 <= 16:
        return _LMHeadCrossEntropy.apply(h, w, targets, V, ignore_index, int(chunk),
                                         bool(signal_w))
    logits = torch.nn.functional.linear(h, w)
    return ref.cross_entropy(logits, targets, V, ignore_index)


class _Embedding(torch.autograd.Function):
    """x = wte[idx] + wpe[:T]; backward scatters straight into the flat gradient sinks
    (fp32 index_add for the token table, a column-batch sum for positions)."""

    @staticmethod
    def forward(ctx, idx, wte, wpe):
        T = idx.shape[1]
        x = torch.nn.functional.embedding(idx, wte) + wpe[:T].unsqueeze(0)
        ctx.save_for_backward(idx)
        ctx.wte, ctx.wpe = wte, wpe
        return x

    @staticmethod
    def backward(ctx, dx):
        (idx,) = ctx.saved_tensors
        wte, wpe = ctx.wte, ctx.wpe
        B, T, C = dx.shape
        d2 = dx.reshape(-1, C)
        sw, sp = _grad_sink(wte), _grad_sink(wpe)
        if (sw is not None and sp is not None and dx.is_cuda and dx.dtype == torch.bfloat16
                and sw.dtype == torch.float32 and sp.dtype == torch.float32 and C % 8 == 0
                and sw.is_contiguous() and sp.is_contiguous() and sp.shape[0] >= T):
            # one HIP pass: scatter-add into the token table, batch-sum into positions
            ev = getattr(wte, "_ra_sink_event", None)
            if ev is not None:  # the LM head's side-stream dW accumulation comes first
                torch.cuda.current_stream(dx.device).wait_event(ev)
                wte._ra_sink_event = None
            ids = idx.reshape(-1)
            ids = ids if ids.dtype == torch.int64 and ids.is_contiguous() else \
                ids.long().contiguous()
            d2c = d2.contiguous()
            # V = the table's row count (the sink may be a flat 1-D view of V*C floats).
            # Out-of-range ids never get here: F.embedding in the forward device-asserts on
            # them, as torch's index_add_ would; the kernel's bound check is a guard only.
            check(_lib.lib().ra_embed_bwd(ptr(d2c), ptr(ids), ptr(sw), ptr(sp), B, T, C,
                                          wte.shape[0], stream_ptr()), "embed_bwd")
            _grad_done(wte)
            _grad_done(wpe)
            return None, None, None
        outs = []
        for p, fill in ((wte, lambda acc: acc.index_add_(0, idx.reshape(-1),
                                                         d2.to(acc.dtype))),
                        (wpe, lambda acc: acc[:T].add_(dx.float().sum(0).to(acc.dtype)))):
            sink = _grad_sink(p)
            if sink is not None:
                ev = getattr(p, "_ra_sink_event", None)
                if ev is not None:  # the LM head's side-stream dW accumulation comes first
                    torch.cuda.current_stream(dx.device).wait_event(ev)
                    p._ra_sink_event = None
                fill(sink)
                _grad_done(p)
                outs.append(None)
            else:
                acc = torch.zeros(p.shape, device=p.device, dtype=torch.float32)
                fill(acc)
                outs.append(acc.to(p.dtype))
        return None, outs[0], outs[1]


def embedding(idx, wte, wpe):
    """Token + learned position embedding for [B, T] indices.

    The direct-sink path is taken under the same condition as the HIP LM head
    (bf16 on the GPU): a tied ``wte`` must receive ALL its gradient contributions
    through sinks, or the DDP readiness signal would fire before autograd's part."""
    if _hip(idx) and wte.dtype == torch.bfloat16 and \
            (getattr(wte, "_ra_direct_grad", False) or getattr(wpe, "_ra_direct_grad", False)):
        return _Embedding.apply(idx, wte, wpe)
    T = idx.shape[1]
    return torch.nn.functional.embedding(idx, wte) + wpe[:T].unsqueeze(0)


def cross_entropy(logits, targets, vocab_size=None, ignore_index=-100):
    """Mean token cross-entropy. ``logits`` may be vocab-padded; columns >= vocab_size are
    excluded from the softmax."""
    V = vocab_size or logits.shape[-1]
    if _hip(logits) and logits.dtype == torch.bfloat16 and logits.shape[-1] % 8 == 0:
        return _CrossEntropy.apply(logits, targets, V, ignore_index)
    return ref.cross_entropy(logits, targets, V, ignore_index)


# --------------------------------------------------------------------- RL kernels
def gae(rewards, values, dones, bootstrap, gamma=0.99, lam=0.95):
    """Time-major [T,B] GAE → (advantages, value_targets), fp32."""
    if not _hip(rewards):
        return ref.gae(rewards, values, dones, bootstrap, gamma, lam)
    T, B = rewards.shape
    r, v, d, bs = (x.float().contiguous() for x in (rewards, values, dones, bootstrap))
    adv = torch.empty_like(r)
    vt = torch.empty_like(r)
    check(_lib.lib().ra_gae(ptr(r), ptr(v), ptr(d), ptr(bs), ptr(adv), ptr(vt), T, B, gamma, lam,
                            stream_ptr()), "gae")
    return adv, vt


def vtrace(log_rhos, discounts, rewards, values, bootstrap, clip_rho=1.0, clip_c=1.0,
           clip_pg_rho=1.0, lam=1.0):
    """Time-major [T,B] V-trace → (vs, pg_advantages), fp32."""
    if not _hip(values):
        return ref.vtrace(log_rhos, discounts, rewards, values, bootstrap, clip_rho, clip_c,
                          clip_pg_rho, lam)
    T, B = values.shape
    lr, dc, r, v, bs = (x.float().contiguous() for x in
                        (log_rhos, discounts, rewards, values, bootstrap))
    vs = torch.empty_like(v)
    pg = torch.empty_like(v)
    check(_lib.lib().ra_vtrace(ptr(lr), ptr(dc), ptr(r), ptr(v), ptr(bs), ptr(vs), ptr(pg), T, B,
                               clip_rho, clip_c, clip_pg_rho, lam, stream_ptr()), "vtrace")
    return vs, pg


def _ppo_grads_bwd(ctx, g):
    """(dlogits, dvpred) = g * the fp32 gradients the fused loss kernel wrote; bf16 heads
    get both in ONE scale-and-cast launch over the concatenated buffer."""
    (grad,) = ctx.saved_tensors
    N, A = ctx.shape
    ldt, vdt = ctx.dtypes
    if grad.is_cuda and ldt == torch.bfloat16 and vdt in (None, torch.bfloat16):
        out = torch.empty(grad.numel(), device=grad.device, dtype=torch.bfloat16)
        check(_lib.lib().ra_scale_to_bf16(ptr(grad), grad.numel(), ptr(g.float().contiguous()),
                                          ptr(out), stream_ptr()), "scale_to_bf16")
    else:
        out = grad * g
    dlog = out[:N * A].view(N, A).to(ldt)
    dvp = out[N * A:].to(vdt) if ctx.has_v else None
    return dlog, dvp


def _ppo_heads(logits, vpred):
    """Kernel inputs for the policy heads: bf16 read directly, anything else as fp32."""
    bf = logits.dtype == torch.bfloat16 and (vpred is None or vpred.dtype == torch.bfloat16)
    cast = (lambda t: t.contiguous()) if bf else (lambda t: t.float().contiguous())
    return cast(logits), (cast(vpred) if vpred is not None else None), int(bf)


class _PPOLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, vpred, old_logits, actions, old_logp, adv, vtarg, hp):
        N, A = logits.shape
        has_v = vpred is not None
        lg, vp, bf = _ppo_heads(logits, vpred)
        grad = torch.empty(N * A + N, device=logits.device, dtype=torch.float32)
        stats = torch.empty(6, device=logits.device, dtype=torch.float32)
        ol = old_logits.float().contiguous() if old_logits is not None else None
        check(_lib.lib().ra_ppo_loss(
            ptr(lg), ptr(ol), ptr(actions.long().contiguous()), ptr(old_logp.float().contiguous()),
            ptr(adv.float().contiguous()), ptr(vp), ptr(vtarg.float().contiguous()) if has_v else None,
            ptr(grad), ptr(grad[N * A:]) if has_v else None, ptr(stats), N, A, hp[0], hp[1], hp[2],
            hp[3], hp[4], bf, stream_ptr()), "ppo_loss")
        ctx.save_for_backward(grad)
        ctx.has_v = has_v
        ctx.shape = (N, A)
        ctx.dtypes = (logits.dtype, vpred.dtype if has_v else None)
        ctx.mark_non_differentiable(stats)
        return stats[0].clone(), stats

    @staticmethod
    def backward(ctx, g, _gs):
        dlog, dvp = _ppo_grads_bwd(ctx, g)
        return dlog, dvp, None, None, None, None, None, None


def ppo_loss(logits, old_logits, actions, old_logp, adv, vpred, vtarg, clip=0.2, vf_clip=10.0,
             vf_coeff=1.0, ent_coeff=0.0, kl_coeff=0.0):
    """Fused PPO loss: returns (total_loss, stats[6] = total, policy, vf, entropy, kl, clipfrac).
    The kernel computes the loss AND its gradient wrt logits/values in one pass."""
    if not _hip(logits) or logits.shape[-1] > 64:
        return ref.ppo_loss(logits, old_logits, actions, old_logp, adv, vpred, vtarg, clip,
                            vf_clip, vf_coeff, ent_coeff, kl_coeff)
    hp = (float(clip), float(vf_clip), float(vf_coeff), float(ent_coeff), float(kl_coeff))
    return _PPOLoss.apply(logits, vpred, old_logits, actions, old_logp, adv, vtarg, hp)


def ppo_pack(old_logits, actions, old_logp, adv, vtarg):
    """The behaviour-side PPO fields of a whole train batch as ONE fp32 table
    [N, A+4] = [old_logits | action | old_logp | adv | vtarg] for ``ppo_loss_packed``
    (actions are exact in fp32 below 2^24)."""
    return torch.cat([old_logits.float(), actions.float().unsqueeze(1), old_logp.float()[:, None],
                      adv.float()[:, None], vtarg.float()[:, None]], 1).contiguous()


class _PPOLossPacked(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, vpred, aux, idx, stats, hp, has_old, inv_n, kl_dev):
        N, A = logits.shape
        lg, vp, bf = _ppo_heads(logits, vpred)
        grad = torch.empty(N * A + N, device=logits.device, dtype=torch.float32)
        check(_lib.lib().ra_ppo_loss_packed(
            ptr(lg), ptr(vp), ptr(aux), aux.shape[1], int(has_old), ptr(idx), ptr(grad),
            ptr(grad[N * A:]), ptr(stats), N, A, hp[0], hp[1], hp[2], hp[3], hp[4],
            ptr(kl_dev), bf, float(inv_n), stream_ptr()), "ppo_loss_packed")
        ctx.save_for_backward(grad)
        ctx.has_v = True
        ctx.shape = (N, A)
        ctx.dtypes = (logits.dtype, vpred.dtype)
        # backward handle only: the loss values are accumulated into `stats`
        return logits.new_empty((), dtype=torch.float32)

    @staticmethod
    def backward(ctx, g):
        dlog, dvp = _ppo_grads_bwd(ctx, g)
        return dlog, dvp, None, None, None, None, None, None, None


def ppo_loss_packed(logits, vpred, aux, idx, stats, clip=0.2, vf_clip=10.0, vf_coeff=1.0,
                    ent_coeff=0.0, kl_coeff=0.0, has_old=True, inv_n=None, kl_dev=None):
    """Fused PPO loss over a minibatch whose behaviour fields are rows ``idx`` of the packed
    table ``aux`` (``ppo_pack``): no gather kernels. The six statistics (means over the
    minibatch, or scaled by ``inv_n``) are ACCUMULATED into ``stats``; the returned scalar
    is a backward handle whose value is undefined (gradients are exact). ``kl_dev``: an
    optional 1-element fp32 device tensor holding the KL coefficient (read at run time, so
    a captured HIP graph stays valid when it changes). GPU only."""
    if not _hip(logits) or logits.shape[-1] > 64:
        raise ValueError("ppo_loss_packed needs HIP tensors and at most 64 actions")
    N = logits.shape[0]
    hp = (float(clip), float(vf_clip), float(vf_coeff), float(ent_coeff), float(kl_coeff))
    return _PPOLossPacked.apply(logits, vpred, aux, idx, stats, hp, has_old,
                                1.0 / N if inv_n is None else inv_n, kl_dev)


class _PPOHeadsLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, wpi, bpi, wvf, bvf, aux, idx, stats, hp, kl_dev, inv_n, has_old):
        N, F = h.shape
        A = wpi.shape[0]
        d7 = torch.empty(N, A + 1, device=h.device, dtype=torch.float32)
        check(_lib.lib().ra_ppo_heads_fwd(
            ptr(h), F, ptr(wpi), ptr(bpi), ptr(wvf), ptr(bvf), ptr(aux), aux.shape[1],
            int(has_old), ptr(idx), ptr(d7), ptr(stats), N, A, hp[0], hp[1], hp[2], hp[3], hp[4],
            ptr(kl_dev), float(inv_n), stream_ptr()), "ppo_heads_fwd")
        ctx.save_for_backward(h, wpi, wvf, d7)
        ctx.params = (wpi, bpi, wvf, bvf)
        return h.new_empty((), dtype=torch.float32)  # backward handle (stats hold the loss)

    @staticmethod
    def backward(ctx, g):
        h, wpi, wvf, d7 = ctx.saved_tensors
        N, F = h.shape
        A = wpi.shape[0]
        L = _lib.lib()
        dh = torch.empty_like(h)
        work = torch.empty(L.ra_ppo_heads_work(A, F), device=h.device, dtype=torch.float32)
        sinks = [_grad_sink(p) for p in ctx.params]
        use_sink = all(t is not None for t in sinks) and len({t.dtype for t in sinks}) == 1
        if use_sink:
            outs = sinks
            flags = 1 | (2 * _sink_f32(sinks[0]))
        else:
            outs = [torch.empty_like(p) for p in ctx.params]
            flags = 2 * _sink_f32(outs[0])
        check(L.ra_ppo_heads_bwd(ptr(h), F, ptr(wpi), ptr(wvf), ptr(d7),
                                 ptr(g.float().contiguous()), ptr(dh), ptr(work), ptr(outs[0]),
                                 ptr(outs[1]), ptr(outs[2]), ptr(outs[3]), flags, N, A,
                                 stream_ptr()), "ppo_heads_bwd")
        if use_sink:
            for p in ctx.params:
                _grad_done(p)
            outs = [None] * 4
        return (dh, *outs, None, None, None, None, None, None, None)


def ppo_heads_supported(h, wpi, bpi, wvf, bvf) -> bool:
    ok = (_hip(h) and h.dim() == 2 and h.dtype == torch.bfloat16 and h.is_contiguous()
          and h.shape[1] % 8 == 0 and h.shape[1] <= 1024 and wpi.shape[0] <= 18)
    return ok and all(t.dtype == torch.bfloat16 and t.is_contiguous()
                      for t in (wpi, bpi, wvf, bvf)) and wvf.numel() == h.shape[1]


def ppo_heads_loss(h, wpi, bpi, wvf, bvf, aux, idx, stats, clip=0.2, vf_clip=10.0, vf_coeff=1.0,
                   ent_coeff=0.0, kl_coeff=0.0, has_old=True, inv_n=None, kl_dev=None):
    """Policy + value heads fused with the PPO loss over a shared encoder output h [N, F]:
    logits = h Wpi^T + bpi, v = h wvf + bvf, the PPO loss of each row (behaviour fields
    gathered from the packed table ``aux`` by ``idx``, statistics ACCUMULATED into
    ``stats``), and a backward producing dh and the four head gradients (written into the
    flat-buffer sinks). Returns a backward handle (value undefined). GPU only."""
    if not ppo_heads_supported(h, wpi, bpi, wvf, bvf):
        raise ValueError("ppo_heads_loss: unsupported shapes/dtypes")
    hp = (float(clip), float(vf_clip), float(vf_coeff), float(ent_coeff), float(kl_coeff))
    return _PPOHeadsLoss.apply(h, wpi, bpi, wvf, bvf, aux, idx, stats, hp, kl_dev,
                               1.0 / h.shape[0] if inv_n is None else inv_n, has_old)


# --------------------------------------------------------------------- bias + ReLU
def _nhwc_rows(t):
    """[M, C] row view of a 2-D tensor or a channels-last NCHW tensor (None if neither)."""
    if t.dim() == 2:
        return t if t.is_contiguous() else None
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])
    return None


def _relu_bias_bwd(dy, y, bias):
    """dh = dy * (y > 0) and the bias gradient (written into the flat sink, returning None,
    or returned) for a ReLU output y in [M, C] row layout (2-D or channels-last)."""
    if _nhwc_rows(dy) is None:
        dy = dy.contiguous(memory_format=torch.channels_last) if dy.dim() == 4 \
            else dy.contiguous()
    dy2, y2 = _nhwc_rows(dy), _nhwc_rows(y)
    M, C = y2.shape
    L = _lib.lib()
    dh = torch.empty_like(y)
    work = torch.empty(L.ra_relu_bwd_work(M, C), device=y.device, dtype=torch.float32)
    sink = _grad_sink(bias)
    db = sink if sink is not None else torch.empty_like(bias)
    flags = (1 if sink is not None else 0) | (2 * _sink_f32(db))
    check(L.ra_relu_bwd_bias(ptr(dy2), ptr(y2), ptr(_nhwc_rows(dh)), ptr(db), ptr(work), M, C,
                             flags, stream_ptr()), "relu_bwd_bias")
    if sink is not None:
        _grad_done(bias)
        return dh, None
    return dh, db


class _BiasReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, bias):
        h2 = _nhwc_rows(h)
        y = torch.empty_like(h)  # keeps channels-last strides
        y2 = _nhwc_rows(y)
        check(_lib.lib().ra_bias_relu_fwd(ptr(h2), ptr(bias), ptr(y2), h2.shape[0], h2.shape[1],
                                          stream_ptr()), "bias_relu_fwd")
        ctx.save_for_backward(y)
        ctx.bias = bias
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return _relu_bias_bwd(dy, y, ctx.bias)


class _LinearReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        y = torch.empty((x.shape[0], w.shape[0]), device=x.device, dtype=x.dtype)
        torch.mm(x, w.t(), out=y)
        check(_lib.lib().ra_bias_relu_fwd(ptr(y), ptr(b), ptr(y), y.shape[0], y.shape[1],
                                          stream_ptr()), "bias_relu_fwd")
        ctx.save_for_backward(x, w, y)
        ctx.bias = b
        ctx.weight = w
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dh, db = _relu_bias_bwd(dy, y, ctx.bias)
        dx = torch.mm(dh, w) if ctx.needs_input_grad[0] else None
        sink = _grad_sink(ctx.weight)
        if sink is not None and sink.is_contiguous():
            sink.addmm_(dh.t(), x)  # weight gradient accumulated straight into the flat buffer
            _grad_done(ctx.weight)
            return dx, None, db
        return dx, torch.mm(dh.t(), x), db


def linear_relu(x, w, b):
    """relu(x @ w.T + b) for 2-D bf16 x: hipBLASLt GEMM + one fused bias/ReLU pass; the
    backward fuses the ReLU mask with the bias-gradient reduction and accumulates the
    weight gradient into the flat-buffer sink (no separate AccumulateGrad)."""
    F_ = w.shape[0]
    if (_hip(x) and x.dim() == 2 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and b is not None and b.dtype == torch.bfloat16 and F_ % 8 == 0
            and 256 % (F_ // 8) == 0 and x.shape[0] > 0):
        return _LinearReLU.apply(x.contiguous(), w, b)
    return torch.relu(torch.nn.functional.linear(x, w, b))


def bias_relu(h, bias):
    """relu(h + bias) over the channel axis (last dim of a 2-D tensor, dim 1 of a
    channels-last NCHW conv output): one fused pass forward, and ONE pass backward that
    also reduces the bias gradient (instead of add + relu + threshold_backward + sum)."""
    C = h.shape[1] if h.dim() == 4 else h.shape[-1]
    if (_hip(h) and h.dtype == torch.bfloat16 and bias is not None
            and bias.dtype == torch.bfloat16 and C % 8 == 0 and 256 % (C // 8) == 0
            and _nhwc_rows(h) is not None and h.numel() > 0):
        return _BiasReLU.apply(h, bias)
    if bias is not None:
        h = h + (bias.view(1, -1, 1, 1) if h.dim() == 4 else bias).to(h.dtype)
    return torch.relu(h)


# --------------------------------------------------------------------- conv + bias + ReLU
def _is_ohwi(w):
    return w.dim() == 4 and w.permute(0, 2, 3, 1).is_contiguous()


class _ConvBiasReLU(torch.autograd.Function):
    """relu(conv2d(x, w, stride) + b) on the conv.hip MFMA kernels. x is a bf16
    channels-last NCHW activation, or the uint8 NHWC frame batch (rows ``idx``, scaled by
    ``scale`` while loading). Backward: one fused ReLU-mask + bias-gradient pass, the
    MFMA weight-gradient kernel (written straight into the flat gradient buffer), and the
    input gradient on MIOpen (only when x is a differentiable activation)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, idx, scale):
        u8 = x.dtype == torch.uint8
        if u8:
            xh = x
            B = idx.shape[0] if idx is not None else x.shape[0]
            H, W, C = x.shape[1:]
        else:
            xh = x.permute(0, 2, 3, 1)
            B, C, H, W = x.shape
        O, I, KH, KW = w.shape
        OH, OW = (H - KH) // stride + 1, (W - KW) // stride + 1
        y = torch.empty((B, OH, OW, O), device=x.device, dtype=torch.bfloat16).permute(0, 3, 1, 2)
        check(_lib.lib().ra_conv_fwd(ptr(xh), ptr(idx), int(u8), ptr(w), ptr(b), ptr(y), B, H, W,
                                     C, KH, KW, stride, O, float(scale), 1, stream_ptr()),
              "conv_fwd")
        ctx.save_for_backward(x, w, y, idx)
        ctx.geom = (u8, B, H, W, C, KH, KW, stride, O, float(scale))
        ctx.bias = b
        ctx.weight = w
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y, idx = ctx.saved_tensors
        u8, B, H, W, C, KH, KW, S, O, scale = ctx.geom
        dh, db = _relu_bias_bwd(dy, y, ctx.bias)
        L = _lib.lib()
        work = torch.empty(L.ra_conv_wgrad_work(B, H, W, C, KH, KW, S, O), device=dy.device,
                           dtype=torch.float32)
        sink = _grad_sink(ctx.weight)
        if sink is not None and not _is_ohwi(sink):
            sink = None
        dw = sink if sink is not None else torch.empty(
            (O, KH, KW, C), device=dy.device, dtype=w.dtype).permute(0, 3, 1, 2)
        flags = (1 if sink is not None else 0) | (2 * _sink_f32(dw))
        xh = x if u8 else x.permute(0, 2, 3, 1)

        def wgrad():
            check(L.ra_conv_wgrad(ptr(xh), ptr(idx), int(u8), ptr(_nhwc_rows(dh)), ptr(work),
                                  work.numel(), ptr(dw), flags, B, H, W, C, KH, KW, S, O, scale,
                                  stream_ptr()), "conv_wgrad")

        # on the main stream: a side-stream conv wgrad measured slower inside the PPO
        # learner's HIP graph (46.3 vs 41.3 ms/update)
        wgrad()
        if sink is not None:
            _grad_done(ctx.weight)
            dw = None
        dx = None
        if not u8 and ctx.needs_input_grad[0]:
            if L.ra_conv_dgrad_supported(KH, KW, C, S, O):
                dxh = torch.empty((B, H, W, C), device=dy.device, dtype=torch.bfloat16)
                check(L.ra_conv_dgrad(ptr(_nhwc_rows(dh)), ptr(w), ptr(dxh), B, H, W, C, KH, KW,
                                      S, O, stream_ptr()), "conv_dgrad")
                dx = dxh.permute(0, 3, 1, 2)
            else:
                dx = torch.ops.aten.convolution_backward(dh, x, w, None, [S, S], [0, 0], [1, 1],
                                                         False, [0, 0], 1,
                                                         [True, False, False])[0]
        return dx, dw, db, None, None, None


def conv2d_bias_relu(x, w, b, stride, idx=None, scale=1.0 / 255.0):
    """relu(conv2d(x, w, b, stride)) (no padding) for the Nature-CNN layer shapes on the
    MFMA kernels; other shapes / devices fall back to MIOpen + ``bias_relu``.

    x: bf16 channels-last NCHW activations, or uint8 NHWC frames (the first layer: rows
    ``idx`` of the batch, multiplied by ``scale``). Returns channels-last NCHW bf16."""
    u8 = x.dtype == torch.uint8
    ok = (_hip(x) and w.dtype == torch.bfloat16 and b is not None and b.dtype == torch.bfloat16
          and _is_ohwi(w) and (idx is None or u8))
    if ok:
        if u8:
            ok = x.dim() == 4 and x.is_contiguous() and x.shape[3] == w.shape[1]
        else:
            ok = x.dtype == torch.bfloat16 and _nhwc_rows(x) is not None and x.shape[1] == w.shape[1]
    if ok:  # the kernels index the input with 32-bit element offsets
        O, I, KH, KW = w.shape
        ok = x.numel() < 2 ** 31 and bool(_lib.lib().ra_conv_supported(KH, KW, I, stride, O,
                                                                          int(u8)))
    if ok and x.shape[0] > 0:
        return _ConvBiasReLU.apply(x, w, b, stride,
                                   idx.long().contiguous() if idx is not None else None, scale)
    if idx is not None:
        x = x.index_select(0, idx)
    if u8:
        x = (x.float() * scale).to(w.dtype).permute(0, 3, 1, 2)
    return bias_relu(torch.nn.functional.conv2d(x, w, None, stride), b)


def gather_cast_u8(x_u8, idx, scale=1.0 / 255.0):
    """bf16 rows ``x_u8[idx] * scale`` in one pass (no uint8 gather copy)."""
    row = x_u8[0].numel() if x_u8.shape[0] else 0
    if not _hip(x_u8) or row % 16 or not x_u8.is_contiguous():
        return (x_u8.index_select(0, idx).float() * scale).to(torch.bfloat16)
    y = torch.empty((idx.shape[0],) + tuple(x_u8.shape[1:]), dtype=torch.bfloat16,
                    device=x_u8.device)
    check(_lib.lib().ra_gather_cast_u8(ptr(x_u8), ptr(idx.long().contiguous()), ptr(y),
                                       idx.shape[0], row, scale, stream_ptr()), "gather_cast_u8")
    return y


class RunningMeanStd:
    """Running observation normalisation (RLlib MeanStdFilter) with device-side Welford merge."""

    def __init__(self, shape, device="cpu", clip=10.0, eps=1e-8):
        self.shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        D = 1
        for s in self.shape:
            D *= s
        self.D = D
        self.mean = torch.zeros(D, device=device, dtype=torch.float32)
        self.m2 = torch.zeros(D, device=device, dtype=torch.float32)
        self.count = 0
        self.clip = clip
        self.eps = eps

    @property
    def var(self):
        return self.m2 / max(self.count - 1, 1)

    def update(self, x):
        x2 = x.reshape(-1, self.D).float().contiguous()
        N = x2.shape[0]
        if N == 0:
            return
        if x2.is_cuda:
            L = _lib.lib()
            work = torch.empty(2 * L.ra_obsnorm_parts(N) * self.D, device=x2.device)
            check(L.ra_obsnorm_update(ptr(x2), N, self.D, float(self.count), ptr(self.mean),
                                      ptr(self.m2), ptr(work), stream_ptr()), "obsnorm_update")
        else:
            bm = x2.mean(0)
            bm2 = ((x2 - bm) ** 2).sum(0)
            n = self.count + N
            d = bm - self.mean
            self.mean = self.mean + d * N / n
            self.m2 = self.m2 + bm2 + d * d * self.count * N / n
        self.count += N

    def normalize(self, x):
        x2 = x.reshape(-1, self.D).float().contiguous()
        if x2.is_cuda:
            y = torch.empty_like(x2)
            check(_lib.lib().ra_obsnorm_apply(ptr(x2), ptr(y), ptr(self.mean), ptr(self.m2),
                                              x2.shape[0], self.D, float(self.count), self.clip,
                                              self.eps, stream_ptr()), "obsnorm_apply")
        else:
            sd = torch.sqrt(torch.clamp(self.var, min=0))
            y = torch.clamp((x2 - self.mean) / (sd + self.eps), -self.clip, self.clip)
        return y.view(x.shape)

    def __call__(self, x, update=True):
        if update:
            self.update(x)
        return self.normalize(x)

    def state_dict(self):
        return {"mean": self.mean.cpu(), "m2": self.m2.cpu(), "count": self.count}

    def load_state_dict(self, s):
        self.mean = s["mean"].to(self.mean.device)
        self.m2 = s["m2"].to(self.m2.device)
        self.count = s["count"]


# --------------------------------------------------------------------- Data preprocessing
def image_normalize(x_u8_nhwc, mean, std, out_dtype=torch.float32):
    """uint8 NHWC → normalised NCHW (fp32 or bf16)."""
    if not _hip(x_u8_nhwc):
        return ref.image_normalize(x_u8_nhwc, mean, std, out_dtype)
    import ctypes

    N, H, W, C = x_u8_nhwc.shape
    if C > 4:
        return ref.image_normalize(x_u8_nhwc, mean, std, out_dtype)
    mean = [float(v) for v in (mean if hasattr(mean, "__len__") else [mean] * C)]
    std = [float(v) for v in (std if hasattr(std, "__len__") else [std] * C)]
    m = (ctypes.c_float * 4)(*(mean + [0.0] * (4 - len(mean))))
    s = (ctypes.c_float * 4)(*(std + [1.0] * (4 - len(std))))
    x = x_u8_nhwc.contiguous()
    y = torch.empty((N, C, H, W), dtype=out_dtype, device=x.device)
    check(_lib.lib().ra_image_normalize(ptr(x), ptr(y), N, H, W, C, ctypes.addressof(m),
                                        ctypes.addressof(s),
                                        1 if out_dtype == torch.bfloat16 else 0, stream_ptr()),
          "image_normalize")
    return y


def resize_bilinear(x_nchw, size):
    OH, OW = size
    if not _hip(x_nchw) or x_nchw.dtype not in (torch.float32, torch.bfloat16):
        return torch.nn.functional.interpolate(x_nchw.float(), size=size, mode="bilinear",
                                               align_corners=False).to(x_nchw.dtype)
    N, C, H, W = x_nchw.shape
    y = torch.empty((N, C, OH, OW), dtype=x_nchw.dtype, device=x_nchw.device)
    check(_lib.lib().ra_resize_bilinear(ptr(x_nchw.contiguous()), ptr(y), N * C, H, W, OH, OW,
                                        1 if x_nchw.dtype == torch.bfloat16 else 0, stream_ptr()),
          "resize_bilinear")
    return y


def cast_scale_u8(x_u8, scale=1.0 / 255.0):
    """uint8 → bf16 * scale (Atari frame scaling)."""
    if not _hip(x_u8) or x_u8.numel() % 8:
        return (x_u8.float() * scale).to(torch.bfloat16)
    y = torch.empty(x_u8.shape, dtype=torch.bfloat16, device=x_u8.device)
    check(_lib.lib().ra_cast_scale_u8(ptr(x_u8.contiguous()), ptr(y), x_u8.numel(), scale,
                                      stream_ptr()), "cast_scale_u8")
    return y
