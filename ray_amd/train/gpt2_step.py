"""One GPT-2 DDP training step on MI355X — the per-worker body of the headline
Ray Train benchmark (TorchTrainer GPT-2-small DDP bf16).

Used by ``ray_amd.train.examples.gpt2.train_func`` (one rank per GPU as
TorchTrainer worker actors — what ``bench.py`` runs) and by ``bench.py --no-ray``
(the same step in a bare torch.distributed.run loop, for comparison). Everything inside ``step()`` is real work: forward, backward, bucketed
RCCL all-reduce overlapped with backward, global-norm clip, fused AdamW.
"""

from __future__ import annotations

import torch
import torch.distributed as dist

from ray_amd.models.gpt2 import GPT2, GPT2Config
from ray_amd.parallel.flat import FlatAdamW, FlatDDP, FlatParams, cosine_lr


class GPT2Trainer:
    """grad_dtype: fp32 (default — the precision torch DDP reduces in) or bf16 (explicit
    gradient compression: half the all-reduce bytes, bf16-rounded accumulation).
    ddp_always_hook: run the bucket hooks / comm stream / RCCL launches even on a world-1
    group (measures the DDP overlap machinery on one GPU)."""

    def __init__(self, cfg: GPT2Config, micro_batch: int, seq_len: int, device,
                 lr: float = 6e-4, bucket_mb: float = 32.0, total_steps: int = 1000,
                 warmup_steps: int = 10, seed: int = 1234, grad_accum: int = 1,
                 grad_dtype: torch.dtype = torch.float32, param_dtype: torch.dtype | None = None,
                 lm_head_chunk: int = 8192, ddp_always_hook: bool = False):
        torch.manual_seed(seed)
        self.cfg = cfg
        self.B, self.T = micro_batch, seq_len
        self.device = torch.device(device)
        self.grad_accum = grad_accum
        if param_dtype is None:  # bf16 compute on the GPU; fp32 for CPU (gloo) runs
            param_dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        model = GPT2(cfg).to(device=self.device, dtype=param_dtype)
        model.lm_head_chunk = lm_head_chunk
        self.model = model
        from ray_amd.ops import functional as rf

        # the block linear weights keep a W^T copy refreshed by the fused AdamW pass (the
        # input-gradient GEMMs read it; no per-weight transpose kernels beside the forward)
        import os

        flat_wt = rf._DGRAD_WT and os.environ.get("RAY_AMD_FLAT_WT", "1") == "1"
        transpose = (lambda n, p: n.endswith("_w")) if flat_wt else None
        self.flat = FlatParams(model, dtype=param_dtype, grad_dtype=grad_dtype,
                               transpose=transpose)
        self.ddp = FlatDDP(self.flat, bucket_mb=bucket_mb, always_hook=ddp_always_hook)
        # AdamW clears the flat gradient in its own pass (no zero_grad memset per step)
        self.opt = FlatAdamW(self.flat, lr=lr, weight_decay=0.1, max_grad_norm=1.0,
                             grad_scale=self.ddp.grad_scale / grad_accum, zero_grad=True)
        self.base_lr = lr
        self.total_steps = total_steps
        self.warmup = warmup_steps
        self.step_idx = 0
        self.last_loss = None

    def synthetic_batch(self, gen: torch.Generator | None = None):
        x = torch.randint(0, self.cfg.vocab_size, (self.B, self.T + 1), device=self.device,
                          generator=gen)
        return x[:, :-1].contiguous(), x[:, 1:].contiguous()

    # ------------------------------------------------------------------ HIP graph
    def enable_graph(self, batches, warm: int = 2):
        """Capture one whole training step — forward, backward (both compute streams),
        DDP finish, clip and AdamW — as a HIP graph and replay it from then on: the step
        costs one host launch instead of ~1.3k, so the GPU never waits for the Python
        launch path (the eager step had ~2.2 ms of idle launch gaps; profiles/r4).
        lr / Adam bias corrections move to device memory (FlatAdamW.use_device_hyper).
        ``warm`` eager steps run first on the capture stream (per-stream GEMM workspaces,
        kernel choices); they are real training steps. World-1 groups only: a multi-rank
        step keeps the eager path with its overlapped RCCL buckets."""
        if self.device.type != "cuda" or self.ddp.enabled:
            return False
        self._static = [(x.clone(), y.clone()) for x, y in batches]
        self.opt.use_device_hyper()
        cur = torch.cuda.current_stream(self.device)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            for _ in range(warm):
                self._eager_step(self._static)
        cur.wait_stream(s)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            self._graph_loss = self._body(self._static)
        self.opt.step_count -= 1  # capture ran opt.step() on the host, no step happened
        self._graph = g
        return True

    def _body(self, batches):
        """The captured work: identical to an eager step minus the host bookkeeping."""
        loss_sum = None
        for i, (x, y) in enumerate(batches):
            self.ddp.sync = i == len(batches) - 1
            loss = self.model(x, y)
            loss.backward()
            loss_sum = loss.detach() if loss_sum is None else loss_sum + loss.detach()
        self.ddp.finish()
        self.opt.step()
        return loss_sum / len(batches)

    def _eager_step(self, batches):
        lr = cosine_lr(self.step_idx, self.base_lr, self.warmup, self.total_steps)
        if self.opt.hyper is not None:
            self.opt.set_device_hyper(lr, self.opt.step_count + 1)
        self.opt.lr = lr
        self.last_loss = self._body(batches)
        self.step_idx += 1
        return self.last_loss

    def step(self, batches):
        """batches: list of (idx, targets), len == grad_accum."""
        g = getattr(self, "_graph", None)
        if g is not None:
            for (sx, sy), (x, y) in zip(self._static, batches):
                if sx.data_ptr() != x.data_ptr():
                    sx.copy_(x, non_blocking=True)
                    sy.copy_(y, non_blocking=True)
            lr = cosine_lr(self.step_idx, self.base_lr, self.warmup, self.total_steps)
            self.opt.step_count += 1
            self.opt.set_device_hyper(lr, self.opt.step_count)
            g.replay()
            # the replayed AdamW changed the weights through raw pointers: host-side caches
            # keyed on the weights epoch (transposed copies outside the flat W^T views) go
            # stale; the flat W^T views were rewritten by the replay itself
            from ray_amd.ops import functional as rf

            rf.bump_weights_epoch()
            self.flat.mark_wt_fresh()
            self.step_idx += 1
            self.last_loss = self._graph_loss
            return self.last_loss
        # the flat gradient was zeroed by the previous AdamW pass (or at creation)
        loss_sum = None
        for i, (x, y) in enumerate(batches):
            self.ddp.sync = i == len(batches) - 1
            loss = self.model(x, y)
            loss.backward()
            loss_sum = loss.detach() if loss_sum is None else loss_sum + loss.detach()
        self.ddp.finish()
        lr = cosine_lr(self.step_idx, self.base_lr, self.warmup, self.total_steps)
        self.opt.step(lr)
        self.step_idx += 1
        self.last_loss = loss_sum / len(batches)
        return self.last_loss

    def tokens_per_step(self) -> int:
        world = dist.get_world_size() if dist.is_initialized() else 1
        return self.B * self.T * self.grad_accum * world
