"""Flat-buffer data parallelism for MI355X: zero-copy gradient buckets on RCCL/xGMI.

Design (vs torch DDP, which copies grads into bucket buffers and all-reduces fp32):

* All parameters become views into ONE bf16 compute buffer ``p16`` backed by ONE
  fp32 master buffer ``p32``; all gradients are views into ONE buffer ``g`` —
  fp32 by default (the precision torch DDP under AMP reduces in), or bf16 as an
  explicit gradient-compression opt-in (``grad_dtype=torch.bfloat16``, half the
  RCCL bytes). Layout is [decay group | no-decay group], each group in *reverse
  registration order* (≈ the order backward produces gradients).
* Our HIP backward kernels accumulate parameter gradients straight into their
  ``_ra_grad`` views (fp32 math; with the fp32 buffer nothing is ever rounded to
  bf16). Parameters reached through plain PyTorch ops fall back to autograd's
  ``.grad`` and a post-accumulate hook adds it into the flat buffer.
* ``g`` is cut into buckets (default 32 MiB, sized for ring all-reduce over
  7 point-to-point xGMI links: large enough to run each link near its
  ~150 GB/s, small enough that the first bucket starts while backward still
  has most of its work ahead). A ``post_accumulate_grad`` hook counts ready
  params per bucket and launches ``all_reduce`` on the bucket *view* as soon
  as it is full — no packing copy, comm overlapped with backward on RCCL's
  own stream.
* The 1/world averaging is folded into the optimizer's gradient scale, and
  global-norm clipping computes its scale on device, so the whole optimizer
  step is two small reductions + ONE fused AdamW launch (ray_amd.ops optim.hip).

Reference parity: python/ray/train/torch/train_loop_utils.py:prepare_model
(wraps DistributedDataParallel); this module is what ``prepare_model(...,
parallel_strategy="flat")`` uses by default on GPU.
"""

from __future__ import annotations

import functools
import math
from typing import Iterable

import torch
import torch.distributed as dist

from ray_amd.ops import _lib
from ray_amd.ops._lib import check, ptr, stream_ptr

ALIGN = 64  # elements; keeps every view 128-byte aligned for vector loads


def _round(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


class FlatParams:
    def __init__(self, module: torch.nn.Module, dtype=torch.bfloat16,
                 no_decay: callable | None = None, grad_dtype=torch.float32,
                 transpose: callable | None = None):
        """``transpose(name, p) -> bool``: 2-D (decayed) weights that keep a transposed bf16
        copy W^T (``p._ra_wt_view``) refreshed by the fused AdamW kernel itself
        (``ra_adamw_flat_wt``) — the nn.Linear input-gradient GEMM reads it
        (ops.functional._transposed_weight). Those weights go first in the buffer,
        [0, n_wt)."""
        self.module = module
        seen = {}
        for name, p in module.named_parameters():
            if p.requires_grad and id(p) not in seen:
                seen[id(p)] = (name, p)
        params = list(seen.values())
        if no_decay is None:
            no_decay = lambda name, p: p.dim() < 2  # noqa: E731
        dec = [(n, p) for n, p in params if not no_decay(n, p)][::-1]
        nod = [(n, p) for n, p in params if no_decay(n, p)][::-1]
        wt = []
        if transpose is not None and dtype == torch.bfloat16 and dev_is_cuda(params):
            wt = [(n, p) for n, p in dec if p.dim() == 2 and p.shape[1] % 4 == 0
                  and p.is_contiguous() and transpose(n, p)]
            ids = {id(p) for _, p in wt}
            dec = wt + [(n, p) for n, p in dec if id(p) not in ids]
        self.order = dec + nod
        dev = params[0][1].device
        offs = []
        o = 0
        for n, p in dec:
            offs.append(o)
            o += _round(p.numel())
        self.n_decay = o
        for n, p in nod:
            offs.append(o)
            o += _round(p.numel())
        self.numel = o
        self.dtype = dtype
        self.device = dev
        self.p32 = torch.zeros(o, dtype=torch.float32, device=dev)
        self.p16 = torch.zeros(o, dtype=dtype, device=dev) if dtype != torch.float32 else self.p32
        self.grad_dtype = grad_dtype
        self.g = torch.zeros(o, dtype=grad_dtype, device=dev)
        self.offsets = offs
        self.names = [n for n, _ in self.order]
        self.n_wt = sum(_round(p.numel()) for _, p in wt)
        self.pt16 = None
        self.wt_table = None
        self.wt_tiles = 0
        # .grad can alias the flat buffer only when dtypes match; otherwise autograd
        # gradients are folded in by a post-accumulate hook (registered before any DDP
        # readiness hook, so the bucket never launches before the add)
        self.alias_grad = grad_dtype == dtype
        self._fold_hooks = []
        with torch.no_grad():
            for (n, p), off in zip(self.order, offs):
                k = p.numel()
                # a channels-last conv weight keeps its layout (OHWI in the flat buffers):
                # NHWC convolutions then never re-layout the weight or its gradient
                cl = (p.dim() == 4 and not p.is_contiguous()
                      and p.is_contiguous(memory_format=torch.channels_last))
                src = p.detach().permute(0, 2, 3, 1) if cl else p.detach()
                self.p32[off:off + k].copy_(src.reshape(-1).float())
                self.p16[off:off + k].copy_(self.p32[off:off + k])
                p.data = self._view(self.p16, off, p.shape, cl)
                p._ra_grad = self._view(self.g, off, p.shape, cl)
                if self.alias_grad:
                    p.grad = p._ra_grad
                else:
                    p.grad = None
                    self._fold_hooks.append(p.register_post_accumulate_grad_hook(_fold_grad))
                # ray_amd.ops backward kernels accumulate straight into p._ra_grad
                p._ra_direct_grad = True
        if wt:
            self._build_wt(wt)

    def _build_wt(self, wt):
        """pt16 (mirrors [0, n_wt): W^T [C, R] at W's own offset) + the device segment table
        of ra_adamw_flat_wt; the copies start fresh (the optimizer keeps them so)."""
        import numpy as np

        L = _lib.lib()
        if len(wt) > L.ra_wt_max_segments():
            return
        self.pt16 = torch.empty(self.n_wt, dtype=torch.bfloat16, device=self.device)
        segs = np.zeros(len(wt), dtype=[("off", "<i8"), ("R", "<i4"), ("C", "<i4"),
                                        ("tile0", "<i4"), ("tc", "<i4")])
        tile = 0
        with torch.no_grad():
            for i, ((n, p), off) in enumerate(zip(wt, self.offsets)):
                R, C = p.shape
                tr, tc = (R + 63) // 64, (C + 63) // 64
                segs[i] = (off, R, C, tile, tc)
                tile += tr * tc
                view = self.pt16[off:off + R * C].view(C, R)
                view.copy_(p.detach().t())
                p._ra_wt_view = view
        self.wt_tiles = tile
        blob = np.zeros(L.ra_wt_table_bytes(), dtype=np.uint8)
        blob[:4] = np.frombuffer(np.int32(len(wt)).tobytes(), dtype=np.uint8)
        raw = segs.tobytes()
        blob[8:8 + len(raw)] = np.frombuffer(raw, dtype=np.uint8)
        self.wt_table = torch.from_numpy(blob).to(self.device)
        self.wt_params = [p for _, p in wt]
        self.mark_wt_fresh()

    def mark_wt_fresh(self):
        """Record that every W^T copy matches its weight as of now (the validity key that
        ops.functional._transposed_weight checks before trusting the copy)."""
        from ray_amd.ops import functional as rf

        ep = rf.weights_epoch()
        for p in getattr(self, "wt_params", ()):
            p._ra_wt_key = (ep, p._version)
            p._ra_wt_ev = None

    @staticmethod
    def _view(buf, off, shape, channels_last):
        k = math.prod(shape)
        if not channels_last:
            return buf[off:off + k].view(shape)
        o, i, h, w = shape
        return buf[off:off + k].view(o, h, w, i).permute(0, 3, 1, 2)

    def params(self) -> list[torch.nn.Parameter]:
        return [p for _, p in self.order]

    def zero_grad(self):
        self.g.zero_()
        if not self.alias_grad:
            for _, p in self.order:
                p.grad = None

    def sync_master_from_params(self):
        with torch.no_grad():
            self.p32.copy_(self.p16.float())


def dev_is_cuda(params) -> bool:
    return bool(params) and params[0][1].is_cuda


def _fold_grad(p):
    """post-accumulate hook: fold an autograd-produced .grad into the flat buffer."""
    if p.grad is not None:
        with torch.no_grad():
            p._ra_grad.add_(p.grad.to(p._ra_grad.dtype))
        p.grad = None


class FlatDDP:
    """Bucketed, backward-overlapped gradient all-reduce over the flat grad buffer.

    Stream protocol (GPU). Gradients of one bucket come from two compute streams: the
    main stream (LayerNorm/bias/embedding/LM-head kernels) and the weight-gradient side
    stream (``ops.functional._side_stream``). A readiness signal only counts; when a bucket
    is full, an event is recorded on each compute stream and a DEDICATED comm stream waits
    on those events and issues the RCCL ``all_reduce`` (RCCL's internal stream then orders
    itself after the comm stream). Neither compute stream
    ever waits on the other, or on the comm stream, during backward: the only joins are
    in ``finish()``, right before the optimizer consumes the gradients.

    ``always_hook=True`` keeps the whole path (hooks, events, comm stream, RCCL launches)
    live on a world-1 group, so its cost can be measured on one GPU
    (``bench.py --ddp-hooks always``).
    """

    def __init__(self, flat: FlatParams, group=None, bucket_mb: float = 32.0,
                 always_hook: bool = False):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.buckets: list[tuple[int, int]] = []
        self.param_bucket: list[int] = []
        esize = flat.g.element_size()
        cap = max(1, int(bucket_mb * 1024 * 1024 / esize))
        start = 0
        cur_end = 0
        sizes = []
        for i, (n, p) in enumerate(flat.order):
            off = flat.offsets[i]
            end = off + _round(p.numel())
            if end - start > cap and cur_end > start:
                self.buckets.append((start, cur_end))
                start = cur_end
            cur_end = end
            self.param_bucket.append(len(self.buckets))
        self.buckets.append((start, cur_end))
        for b in range(len(self.buckets)):
            sizes.append(sum(1 for x in self.param_bucket if x == b))
        self.bucket_sizes = sizes
        self._ready = [0] * len(self.buckets)
        self._seen = [False] * len(flat.order)
        self._works = []
        self._hooks = []
        self.enabled = self.world > 1 or (always_hook and dist.is_initialized())
        self.sync = True  # False inside gradient-accumulation micro-steps (no_sync)
        self.launched = 0  # all_reduce launches since construction (tests / bench report)
        self.launched_bytes = 0
        # per-step diagnostics (bench.py): per-bucket all-reduce time on the comm stream and
        # the main stream's exposed wait in finish(), as CUDA events read after a sync
        self.stats = False
        self._step_events: list = []  # [(kind, bytes, ev_start, ev_end)]
        cuda = flat.g.is_cuda and self.enabled
        self._comm = torch.cuda.Stream(flat.device) if cuda else None
        # the training loop's stream (backward's main stream); hooks may fire while a side
        # stream is current, so it is named explicitly
        self._main = torch.cuda.current_stream(flat.device) if cuda else None
        # per bucket: {compute-stream index: event}, reused every step
        self._events: list[dict] = [dict() for _ in self.buckets]
        if self.enabled:
            for i, (_, p) in enumerate(flat.order):
                hook = self._make_hook(i)
                self._hooks.append(p.register_post_accumulate_grad_hook(hook))
                # direct-accumulating ops (ray_amd.ops.functional) bypass AccumulateGrad and
                # signal readiness through this callback instead
                p._ra_grad_ready = functools.partial(hook, p)
        # bucket broadcast of initial weights so every rank starts identical
        if self.enabled:
            dist.broadcast(flat.p32, src=0, group=group)
            with torch.no_grad():
                flat.p16.copy_(flat.p32)

    def _compute_streams(self):
        from ray_amd.ops import functional as rf

        dev = self.flat.device
        out, seen = [], set()
        for st in (self._main, torch.cuda.current_stream(dev), rf._side.get(dev)):
            if st is not None and st.cuda_stream not in seen:
                seen.add(st.cuda_stream)
                out.append(st)
        return out

    def _launch(self, b: int):
        s, e = self.buckets[b]
        if self._comm is None:
            work = dist.all_reduce(self.flat.g[s:e], group=self.group, async_op=True)
        else:
            # one event per compute stream (main + weight-gradient side streams), recorded
            # now: it follows every gradient of the bucket those streams produced (their
            # kernels were enqueued before their hooks ran), so the comm stream never
            # starts early; it may wait for a little more of a stream's work than the
            # bucket's gradients, which the overlapped backward hides. Nothing is recorded
            # per parameter: the hooks stay a counter bump (host cost between backward's
            # kernel launches)
            for i, st in enumerate(self._compute_streams()):
                evs = self._events[b]
                ev = evs.get(i)
                if ev is None:
                    ev = evs[i] = torch.cuda.Event()
                ev.record(st)
                self._comm.wait_event(ev)
            with torch.cuda.stream(self._comm):
                if self.stats:
                    ev0 = torch.cuda.Event(enable_timing=True)
                    ev0.record(self._comm)
                work = dist.all_reduce(self.flat.g[s:e], group=self.group, async_op=True)
                if self.stats:
                    # the comm stream waits for the collective: the next bucket's start
                    # event then marks an idle RCCL stream, so (ev0, ev1) is this bucket's
                    # all-reduce time, not queueing behind the previous one
                    work.wait()
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev1.record(self._comm)
                    self._step_events.append(("bucket", (e - s) * self.flat.g.element_size(),
                                              ev0, ev1))
        self._works.append(work)
        self.launched += 1
        self.launched_bytes += (e - s) * self.flat.g.element_size()

    def _make_hook(self, i: int):
        b = self.param_bucket[i]

        def hook(_p):
            # a param can be signalled twice per backward (a direct-accumulating op, then the
            # AccumulateGrad post-hook which PyTorch also runs for a None grad): count once
            if not self.sync or self._seen[i]:
                return
            self._seen[i] = True
            self._ready[b] += 1
            if self._ready[b] == self.bucket_sizes[b]:
                self._launch(b)

        return hook

    def finish(self):
        """Wait (on-stream, no host block) for every bucket; reset counters."""
        if not self.enabled:
            return
        if self.flat.g.is_cuda:
            from ray_amd.ops import functional as rf

            rf.join_side_streams()
        # buckets never triggered (unused params, or params without a readiness signal)
        # are reduced now, after both compute streams joined
        for b, r in enumerate(self._ready):
            if r != self.bucket_sizes[b]:
                s, e = self.buckets[b]
                self._works.append(dist.all_reduce(self.flat.g[s:e], group=self.group,
                                                   async_op=True))
                self.launched += 1
                self.launched_bytes += (e - s) * self.flat.g.element_size()
        t_ev = None
        if self.stats and self.flat.g.is_cuda:
            # recorded after the side-stream join: only the wait for RCCL lies between
            t_ev = torch.cuda.Event(enable_timing=True)
            t_ev.record()
        for w in self._works:
            w.wait()  # the current stream waits on RCCL's stream (no host block)
        if t_ev is not None:
            t_end = torch.cuda.Event(enable_timing=True)
            t_end.record()
            self._step_events.append(("exposed", 0, t_ev, t_end))
        self._works.clear()
        self._ready = [0] * len(self.buckets)
        self._seen = [False] * len(self.flat.order)

    def reset_stats(self):
        self._step_events = []
        self._stats_launched = self.launched
        self._stats_bytes = self.launched_bytes

    def read_stats(self, steps: int) -> dict:
        """Per-step DDP diagnostics since ``reset_stats`` (call after a device sync):
        exposed communication (the main stream's wait for RCCL in finish()), all-reduce
        launches / bytes per step, and per-bucket all-reduce time and bus bandwidth
        (busbw = bytes / t x 2 (n - 1) / n, the ring all-reduce's per-link traffic)."""
        steps = max(1, steps)
        exposed = [a.elapsed_time(b) for k, _, a, b in self._step_events if k == "exposed"]
        buckets = [(n, a.elapsed_time(b)) for k, n, a, b in self._step_events if k == "bucket"]
        n = self.world
        factor = 2.0 * (n - 1) / n if n > 1 else 1.0
        bus = [nb / (ms * 1e-3) / 1e9 * factor for nb, ms in buckets if ms > 0]
        launched = self.launched - getattr(self, "_stats_launched", 0)
        nbytes = self.launched_bytes - getattr(self, "_stats_bytes", 0)
        return {
            "ddp_exposed_comm_ms_per_step": round(sum(exposed) / steps, 4) if exposed else 0.0,
            "ddp_allreduce_launches_per_step": round(launched / steps, 2),
            "ddp_allreduce_mb_per_step": round(nbytes / steps / 2 ** 20, 2),
            "ddp_allreduce_ms_per_step": round(sum(ms for _, ms in buckets) / steps, 4)
            if buckets else 0.0,
            "ddp_bucket_busbw_gbps_mean": round(sum(bus) / len(bus), 2) if bus else None,
            "ddp_bucket_busbw_gbps_min": round(min(bus), 2) if bus else None,
            "ddp_buckets": len(self.buckets),
        }

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world


class FlatAdamW:
    """Fused AdamW over a FlatParams buffer (fp32 master, bf16 compute/grad)."""

    def __init__(self, flat: FlatParams, lr=6e-4, betas=(0.9, 0.95), eps=1e-8,
                 weight_decay=0.1, max_grad_norm: float | None = 1.0, grad_scale: float = 1.0,
                 zero_grad: bool = False):
        self.flat = flat
        self.lr = lr
        self.b1, self.b2 = betas
        self.eps = eps
        self.wd = weight_decay
        self.max_grad_norm = max_grad_norm
        self.grad_scale = grad_scale
        dev = flat.device
        self.m = torch.zeros_like(flat.p32)
        self.v = torch.zeros_like(flat.p32)
        self.step_count = 0
        self._scale = torch.ones(1, dtype=torch.float32, device=dev)
        self.last_norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self._work = None
        self.use_hip = flat.p32.is_cuda
        # clear the gradient inside the AdamW pass (the caller then skips zero_grad)
        self.zero_grad = zero_grad
        # graph-captured steps: {lr, 1/(1-b1^t), 1/(1-b2^t)} live in device memory and are
        # refreshed before every replay (set_device_hyper)
        self.hyper = None
        self._hyper_ring = None

    def use_device_hyper(self):
        """Switch to device-resident lr / bias corrections (HIP-graph capture of step())."""
        dev = self.flat.device
        self.hyper = torch.zeros(4, dtype=torch.float32, device=dev)
        # pinned staging slots, each reusable once its async copy has run
        self._hyper_ring = [(torch.zeros(4, dtype=torch.float32, pin_memory=True),
                             torch.cuda.Event()) for _ in range(8)]
        self._ring_i = 0

    def set_device_hyper(self, lr: float, step: int):
        """Enqueue (on the current stream) the hyper-parameters of optimizer step ``step``."""
        host, ev = self._hyper_ring[self._ring_i % len(self._hyper_ring)]
        self._ring_i += 1
        ev.synchronize()  # the copy that last read this slot has executed
        host[0] = lr
        host[1] = 1.0 / (1.0 - self.b1 ** step)
        host[2] = 1.0 / (1.0 - self.b2 ** step)
        self.hyper.copy_(host, non_blocking=True)
        ev.record()

    def step(self, lr: float | None = None):
        from ray_amd.ops import functional as rf

        if self.use_hip:
            rf.join_side_streams()  # weight gradients queued on the side stream
            rf.bound_run_ahead()
        rf.bump_weights_epoch()  # the kernel updates p16 in place: cached copies go stale
        self.step_count += 1
        lr = self.lr if lr is None else lr
        f = self.flat
        if self.use_hip:
            L = _lib.lib()
            s = stream_ptr()
            gptr = ptr(self._scale)
            if self.max_grad_norm or self.grad_scale != 1.0:
                if self._work is None:
                    self._work = torch.empty(L.ra_norm_parts(), dtype=torch.float32,
                                             device=f.device)
                check(L.ra_grad_clip(ptr(f.g), f.numel, 1 if f.g.dtype == torch.bfloat16 else 0,
                                     float(self.max_grad_norm or 0.0), float(self.grad_scale),
                                     ptr(self._work), gptr, ptr(self.last_norm), s), "grad_clip")
            else:
                gptr = None
            g32 = f.g.dtype == torch.float32
            if f.pt16 is not None:
                # AdamW + the W^T copies of the linear weights in one pass
                check(L.ra_adamw_flat_wt(ptr(f.p32), ptr(f.p16), ptr(f.pt16), ptr(f.g),
                                         ptr(self.m), ptr(self.v), f.numel, f.n_decay, f.n_wt,
                                         ptr(f.wt_table), f.wt_tiles, lr, self.b1, self.b2,
                                         self.eps, self.wd, self.step_count, gptr,
                                         (1 if g32 else 0) | (2 if self.zero_grad else 0),
                                         ptr(self.hyper) if self.hyper is not None else None, s),
                      "adamw_wt")
                f.mark_wt_fresh()
                return
            check(L.ra_adamw_flat_dev(ptr(f.p32), ptr(f.p16) if f.p16 is not f.p32 else None,
                                      ptr(f.g), ptr(self.m), ptr(self.v), f.numel, f.n_decay,
                                      lr, self.b1, self.b2, self.eps, self.wd, self.step_count,
                                      gptr, (1 if g32 else 0) | (2 if self.zero_grad else 0),
                                      ptr(self.hyper) if self.hyper is not None else None, s),
                  "adamw")
            return
        # CPU reference path (same math)
        g = f.g.float() * self.grad_scale
        norm = g.norm()
        self.last_norm.fill_(norm.item())
        if self.max_grad_norm and norm > self.max_grad_norm:
            g = g * (self.max_grad_norm / (norm + 1e-6))
        self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
        self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
        bc1 = 1 - self.b1 ** self.step_count
        bc2 = 1 - self.b2 ** self.step_count
        upd = (self.m / bc1) / ((self.v / bc2).sqrt() + self.eps)
        decay = torch.ones_like(f.p32)
        decay[: f.n_decay] = 1 - lr * self.wd
        f.p32.mul_(decay).sub_(lr * upd)
        if f.p16 is not f.p32:
            f.p16.copy_(f.p32)
        if self.zero_grad:
            f.g.zero_()

    def state_dict(self):
        return {"m": self.m, "v": self.v, "step": self.step_count}

    def load_state_dict(self, s):
        self.m.copy_(s["m"])
        self.v.copy_(s["v"])
        self.step_count = s["step"]


def cosine_lr(step: int, base: float, warmup: int, total: int, min_ratio: float = 0.1) -> float:
    if step < warmup:
        return base * (step + 1) / warmup
    t = min(1.0, (step - warmup) / max(1, total - warmup))
    return base * (min_ratio + (1 - min_ratio) * 0.5 * (1 + math.cos(math.pi * t)))
