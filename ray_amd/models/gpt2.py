"""GPT-2 (small/medium/large/xl) for MI355X, random init.

The headline Ray Train workload (BASELINE.json config 2: TorchTrainer GPT-2-small
DDP bf16). Architecture per Radford et al. 2019 / HF GPT2LMHeadModel (pre-LN,
learned positions, tanh-GELU, tied input/output embedding).

MI355X-first choices:
* bf16 weights/activations end to end (fp32 master lives in the flat optimizer).
* Every GEMM is a plain hipBLASLt GEMM with NO bias; the bias, activation and
  residual are fused into a single HBM pass by our HIP epilogue kernels
  (``bias_gelu``, ``bias_residual``), LayerNorm and the vocab cross-entropy are
  hand-written kernels (ray_amd/ops/csrc).
* Vocab padded 50257 → 50304 (multiple of 64/128) so the LM-head GEMM tiles
  cleanly on MFMA; padded columns are masked inside the fused cross-entropy.
* LM head + cross-entropy fused and chunked over tokens (``lm_head_cross_entropy``):
  the 64x1024x50304 logits tensor (6.6 GB) never exists; each chunk's logits are
  turned into dlogits in place by one register-resident HIP pass.
* Attention: our HIP MFMA causal flash attention (ops/csrc/attn.hip) reading the
  packed QKV GEMM output directly.
* Backward: split-K fp32 weight-gradient GEMMs and every parameter gradient
  (weights, biases, LayerNorm) accumulated in place into the flat DDP gradient
  buffer (no AccumulateGrad adds); the residual stream's two gradients are summed
  inside the LayerNorm backward kernel (``LayerNorm.fork``).
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ray_amd.ops import functional as rf


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    padded_vocab: int = 50304
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    layer_norm_eps: float = 1e-5
    init_std: float = 0.02

    @staticmethod
    def small():
        return GPT2Config()

    @staticmethod
    def medium():
        return GPT2Config(n_embd=1024, n_layer=24, n_head=16)

    @staticmethod
    def large():
        return GPT2Config(n_embd=1280, n_layer=36, n_head=20)

    @staticmethod
    def xl():
        return GPT2Config(n_embd=1600, n_layer=48, n_head=25)

    @staticmethod
    def tiny():
        return GPT2Config(vocab_size=512, padded_vocab=512, n_positions=128, n_embd=64,
                          n_layer=2, n_head=4)


class LayerNorm(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.bias = nn.Parameter(torch.zeros(d))
        self.eps = eps

    def forward(self, x):
        return rf.layer_norm(x, self.weight, self.bias, self.eps)

    def fork(self, x):
        """(x for the residual add, LN(x)) — the residual grads are summed in the LN bwd."""
        return rf.layer_norm_fork(x, self.weight, self.bias, self.eps)


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        C = cfg.n_embd
        self.n_head = cfg.n_head
        self.ln_1 = LayerNorm(C, cfg.layer_norm_eps)
        self.c_attn_w = nn.Parameter(torch.empty(3 * C, C))
        self.c_attn_b = nn.Parameter(torch.zeros(3 * C))
        self.c_proj_w = nn.Parameter(torch.empty(C, C))
        self.c_proj_b = nn.Parameter(torch.zeros(C))
        self.ln_2 = LayerNorm(C, cfg.layer_norm_eps)
        self.c_fc_w = nn.Parameter(torch.empty(4 * C, C))
        self.c_fc_b = nn.Parameter(torch.zeros(4 * C))
        self.mlp_proj_w = nn.Parameter(torch.empty(C, 4 * C))
        self.mlp_proj_b = nn.Parameter(torch.zeros(C))

    def attn(self, h):
        """Attention sub-block on the normalised input; returns the projection output
        WITHOUT its bias (added by the fused residual+LayerNorm seam)."""
        B, T, C = h.shape
        qkv = rf.linear(h, self.c_attn_w, self.c_attn_b)  # + bias epilogue
        # HIP MFMA flash attention straight off the packed QKV layout (no permutes/copies)
        y = rf.causal_attention_qkv(qkv.view(B, T, 3, self.n_head, C // self.n_head))
        return rf.linear(y.reshape(B, T, C), self.c_proj_w)

    def mlp(self, h):
        a = rf.bias_gelu(rf.linear(h, self.c_fc_w), self.c_fc_b)
        return rf.linear(a, self.mlp_proj_w)

    def forward(self, x):
        x, h = self.ln_1.fork(x)
        x = rf.bias_residual(self.attn(h), self.c_proj_b, x)
        x, h = self.ln_2.fork(x)
        return rf.bias_residual(self.mlp(h), self.mlp_proj_b, x)


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.cfg = cfg
        self.wte = nn.Parameter(torch.empty(cfg.padded_vocab, cfg.n_embd))
        self.wpe = nn.Parameter(torch.empty(cfg.n_positions, cfg.n_embd))
        self.h = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = LayerNorm(cfg.n_embd, cfg.layer_norm_eps)
        self.lm_head_chunk = 8192  # tokens per fused LM-head/CE chunk
        self.reset_parameters()

    def reset_parameters(self):
        std = self.cfg.init_std
        proj_std = std / math.sqrt(2 * self.cfg.n_layer)
        with torch.no_grad():
            nn.init.normal_(self.wte, 0, std)
            self.wte[self.cfg.vocab_size:].zero_()
            nn.init.normal_(self.wpe, 0, 0.01)
            for b in self.h:
                nn.init.normal_(b.c_attn_w, 0, std)
                nn.init.normal_(b.c_fc_w, 0, std)
                nn.init.normal_(b.c_proj_w, 0, proj_std)
                nn.init.normal_(b.mlp_proj_w, 0, proj_std)

    def num_params(self, non_embedding=True):
        n = sum(p.numel() for p in self.parameters())
        if non_embedding:
            n -= self.wpe.numel()
        return n

    def forward(self, idx, targets=None):
        B, T = idx.shape
        x = rf.embedding(idx, self.wte, self.wpe)
        # Pre-LN seams fused: every "x += sub_block(h) + bias; h = LN(x)" is ONE kernel
        # forward and ONE kernel backward (residual grads, LN grads and the projection-bias
        # grad together) — see ops.functional.residual_layer_norm.
        x, h = self.h[0].ln_1.fork(x)
        for i, blk in enumerate(self.h):
            x, h = rf.residual_layer_norm(blk.attn(h), blk.c_proj_b, x, blk.ln_2.weight,
                                          blk.ln_2.bias, blk.ln_2.eps)
            nxt = self.h[i + 1].ln_1 if i + 1 < len(self.h) else self.ln_f
            x, h = rf.residual_layer_norm(blk.mlp(h), blk.mlp_proj_b, x, nxt.weight, nxt.bias,
                                          nxt.eps)
        if targets is None:
            logits = F.linear(h, self.wte)  # tied LM head on ln_f(x), [B, T, padded_vocab]
            return logits[..., : self.cfg.vocab_size]
        # tied LM head + CE fused and chunked over tokens (never the full logits); the
        # embedding backward, which runs last, signals wte's DDP readiness
        return rf.lm_head_cross_entropy(h, self.wte, targets, self.cfg.vocab_size,
                                        chunk=self.lm_head_chunk, signal_w=False)

    def flops_per_token(self, T: int) -> float:
        """6N + 12·L·H·hd·T (PaLM appendix B convention), training FLOPs per token."""
        cfg = self.cfg
        N = self.num_params()
        return 6 * N + 12 * cfg.n_layer * cfg.n_embd * T
