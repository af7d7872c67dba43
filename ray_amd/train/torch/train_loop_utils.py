"""Torch helpers for training loops (reference: python/ray/train/torch/train_loop_utils.py).

``prepare_model`` on MI355X: bf16 models on GPU go through the flat-buffer DDP of
``ray_amd.parallel.flat`` (zero-copy bf16 grad buckets all-reduced on RCCL while
backward runs, fused AdamW); any other model is wrapped in torch DDP (gloo on CPU).
"""

from __future__ import annotations

import os
import random

import torch
import torch.distributed as dist


def get_device() -> torch.device:
    if torch.cuda.is_available():
        idx = int(os.environ.get("RAY_AMD_LOCAL_DEVICE", "0"))
        if idx >= torch.cuda.device_count():
            idx = 0
        return torch.device("cuda", idx)
    return torch.device("cpu")


def get_devices():
    return [get_device()]


class FlatPreparedModel(torch.nn.Module):
    """Wrapper returned by prepare_model(parallel_strategy='flat'): the module plus its
    flat parameter/gradient buffers, bucketed all-reduce and fused optimizer."""

    def __init__(self, module, flat, ddp):
        super().__init__()
        self.module = module
        self.flat = flat
        self.ddp = ddp

    def forward(self, *a, **k):
        return self.module(*a, **k)

    def make_optimizer(self, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=1.0):
        from ray_amd.parallel.flat import FlatAdamW

        return _FlatOptimizer(self, FlatAdamW(self.flat, lr=lr, betas=betas,
                                              weight_decay=weight_decay,
                                              max_grad_norm=max_grad_norm,
                                              grad_scale=self.ddp.grad_scale))


class _FlatOptimizer:
    def __init__(self, model: FlatPreparedModel, opt):
        self.model = model
        self.opt = opt

    def zero_grad(self, set_to_none=False):
        self.model.flat.zero_grad()

    def step(self, lr=None):
        self.model.ddp.finish()
        self.opt.step(lr)

    @property
    def param_groups(self):
        return [{"lr": self.opt.lr}]


def prepare_model(model: torch.nn.Module, move_to_device: bool = True,
                  parallel_strategy: str | None = "auto", parallel_strategy_kwargs=None):
    dev = get_device()
    if move_to_device:
        model = model.to(dev)
    kw = parallel_strategy_kwargs or {}
    world = dist.get_world_size() if dist.is_initialized() else 1
    params = list(model.parameters())
    is_bf16 = params and all(p.dtype == torch.bfloat16 for p in params)
    if parallel_strategy == "flat" or (parallel_strategy == "auto" and dev.type == "cuda" and
                                       is_bf16):
        from ray_amd.parallel.flat import FlatDDP, FlatParams

        gd = kw.get("grad_dtype", torch.float32)  # fp32 reduce by default (torch DDP parity)
        flat = FlatParams(model, dtype=params[0].dtype, grad_dtype=gd)
        ddp = FlatDDP(flat, bucket_mb=kw.get("bucket_mb", 32.0))
        return FlatPreparedModel(model, flat, ddp)
    if _AMP["enabled"]:
        # patch forward in place BEFORE the parallel wrapper (reference: train_loop_utils
        # prepare_model with amp): no wrapper module, so state_dict keys are identical with
        # and without AMP and checkpoints load into the plain model
        model.forward = _AutocastForward(model, dev.type, _AMP["dtype"])
    return _wrap_parallel(model, dev, world, parallel_strategy, kw)


def _wrap_parallel(model, dev, world, parallel_strategy, kw):
    if world > 1 and parallel_strategy in ("auto", "ddp"):
        from torch.nn.parallel import DistributedDataParallel as DDP

        if dev.type == "cuda":
            return DDP(model, device_ids=[dev], output_device=dev,
                       bucket_cap_mb=kw.get("bucket_cap_mb", 32), **{k: v for k, v in kw.items()
                                                                    if k != "bucket_cap_mb"})
        return DDP(model, **kw)
    if parallel_strategy == "fsdp" and world > 1:
        from torch.distributed.fsdp import FullyShardedDataParallel as FSDP

        return FSDP(model, device_id=dev if dev.type == "cuda" else None, **kw)
    return model


class _DeviceLoader:
    def __init__(self, loader, device, auto_transfer=True):
        self.loader = loader
        self.device = device
        self.auto = auto_transfer
        self.stream = torch.cuda.Stream(device) if device.type == "cuda" else None

    def _move(self, b):
        if isinstance(b, torch.Tensor):
            return b.to(self.device, non_blocking=True)
        if isinstance(b, (list, tuple)):
            return type(b)(self._move(x) for x in b)
        if isinstance(b, dict):
            return {k: self._move(v) for k, v in b.items()}
        return b

    def __iter__(self):
        it = iter(self.loader)
        if self.stream is None or not self.auto:
            for b in it:
                yield self._move(b) if self.auto else b
            return
        # double-buffered H2D on a side stream (pinned host memory -> HBM overlaps compute)
        nxt = None
        try:
            first = next(it)
        except StopIteration:
            return
        with torch.cuda.stream(self.stream):
            nxt = self._move(first)
        for b in it:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            cur = nxt
            with torch.cuda.stream(self.stream):
                nxt = self._move(b)
            yield cur
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        yield nxt

    def __len__(self):
        return len(self.loader)


def prepare_data_loader(data_loader, add_dist_sampler: bool = True, move_to_device: bool = True,
                        auto_transfer: bool = True):
    from torch.utils.data import DataLoader, DistributedSampler

    if add_dist_sampler and dist.is_initialized() and dist.get_world_size() > 1 and \
            not isinstance(getattr(data_loader, "sampler", None), DistributedSampler):
        shuffle = isinstance(getattr(data_loader, "sampler", None),
                             torch.utils.data.RandomSampler)
        sampler = DistributedSampler(data_loader.dataset, shuffle=shuffle)
        data_loader = DataLoader(data_loader.dataset, batch_size=data_loader.batch_size,
                                 sampler=sampler, num_workers=data_loader.num_workers,
                                 collate_fn=data_loader.collate_fn,
                                 pin_memory=get_device().type == "cuda",
                                 drop_last=data_loader.drop_last)
    if move_to_device:
        return _DeviceLoader(data_loader, get_device(), auto_transfer)
    return data_loader


# accelerate(amp=True) state: models prepared afterwards run their forward under autocast
# (bf16 on MI355X: no loss scaling needed); fp16 autocast adds a GradScaler
_AMP = {"enabled": False, "dtype": torch.bfloat16, "scaler": None}


class _AutocastForward:
    """A module's forward, run under torch.autocast; installed as the instance attribute
    ``forward`` so nn.Module.__call__ (and DDP/FSDP around it) pick it up. Holds the module
    rather than a bound method, so the patched module still pickles."""

    def __init__(self, module, device_type, dtype):
        self.module = module
        self.device_type = device_type
        self.dtype = dtype

    def __call__(self, *a, **k):
        with torch.autocast(self.device_type, dtype=self.dtype):
            return type(self.module).forward(self.module, *a, **k)


class _AmpOptimizer:
    """Optimizer facade for fp16 AMP: step / zero_grad go through the GradScaler
    (reference: train/torch/train_loop_utils.py _WrappedOptimizer)."""

    def __init__(self, optimizer, scaler):
        self.optimizer = optimizer
        self.scaler = scaler

    def step(self, closure=None):
        self.scaler.step(self.optimizer, closure) if closure else self.scaler.step(self.optimizer)
        self.scaler.update()

    def zero_grad(self, set_to_none: bool = True):
        self.optimizer.zero_grad(set_to_none=set_to_none)

    def __getattr__(self, name):
        return getattr(self.optimizer, name)


def prepare_optimizer(optimizer):
    """With accelerate(amp=True) in fp16 mode: wrap for loss scaling; otherwise unchanged
    (bf16 autocast needs no scaler)."""
    if _AMP["enabled"] and _AMP["scaler"] is not None and \
            not isinstance(optimizer, (_AmpOptimizer, _FlatOptimizer)):
        return _AmpOptimizer(optimizer, _AMP["scaler"])
    return optimizer


def backward(tensor):
    """loss.backward(), scaled when fp16 AMP is active."""
    if _AMP["enabled"] and _AMP["scaler"] is not None:
        _AMP["scaler"].scale(tensor).backward()
    else:
        tensor.backward()


def enable_reproducibility(seed: int = 0):
    torch.manual_seed(seed)
    random.seed(seed)
    try:
        import numpy as np

        np.random.seed(seed)
    except ImportError:
        pass
    torch.use_deterministic_algorithms(True, warn_only=True)


def accelerate(amp: bool = False, amp_dtype: str = "bf16"):
    """Enable automatic mixed precision for the models / optimizers prepared after this call
    (reference: ray.train.torch.accelerate). bf16 (default on MI355X) autocasts matmuls to
    bf16 with fp32 master weights; fp16 adds dynamic loss scaling via prepare_optimizer /
    backward."""
    _AMP["enabled"] = bool(amp)
    _AMP["dtype"] = torch.float16 if amp_dtype == "fp16" else torch.bfloat16
    _AMP["scaler"] = None
    if amp and _AMP["dtype"] == torch.float16:
        dev = get_device()
        _AMP["scaler"] = torch.amp.GradScaler(dev.type)
