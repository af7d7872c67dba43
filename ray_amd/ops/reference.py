"""Plain-PyTorch fp32 reference implementations of every HIP kernel.

Used (a) by the numerics tests as ground truth and (b) as the CPU path, so the
whole framework runs on CPU-only hosts. GPU tensors never route here: see
``ray_amd.ops.functional``.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def layer_norm(x, weight, bias, eps=1e-5):
    return F.layer_norm(x.float(), (x.shape[-1],), weight.float(), bias.float(), eps).to(x.dtype)


def gelu_tanh(u):
    return 0.5 * u * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (u + 0.044715 * u.pow(3))))


def bias_gelu(h, bias):
    return gelu_tanh(h.float() + bias.float()).to(h.dtype)


def bias_residual(h, bias, res):
    out = res.float() + h.float()
    if bias is not None:
        out = out + bias.float()
    return out.to(h.dtype)


def cross_entropy(logits, targets, vocab_size=None, ignore_index=-100):
    V = vocab_size or logits.shape[-1]
    lf = logits[..., :V].float().reshape(-1, V)
    return F.cross_entropy(lf, targets.reshape(-1), ignore_index=ignore_index)


def _f(x):
    return x.to(torch.promote_types(x.dtype, torch.float32))


def gae(rewards, values, dones, bootstrap, gamma, lam):
    """[T,B] time-major GAE. Returns (advantages, value_targets)."""
    rewards, values, dones, bootstrap = map(_f, (rewards, values, dones, bootstrap))
    T = rewards.shape[0]
    adv = torch.zeros_like(rewards)
    last = torch.zeros_like(bootstrap)
    vnext = bootstrap
    for t in range(T - 1, -1, -1):
        nt = 1.0 - dones[t]
        delta = rewards[t] + gamma * vnext * nt - values[t]
        last = delta + gamma * lam * nt * last
        adv[t] = last
        vnext = values[t]
    return adv, adv + values


def vtrace(log_rhos, discounts, rewards, values, bootstrap, clip_rho=1.0, clip_c=1.0,
           clip_pg_rho=1.0, lam=1.0):
    """Time-major V-trace (Espeholt et al. 2018). Returns (vs, pg_advantages)."""
    log_rhos, discounts, rewards, values, bootstrap = map(
        _f, (log_rhos, discounts, rewards, values, bootstrap))
    rhos = torch.exp(log_rhos)
    crho = torch.clamp(rhos, max=clip_rho)
    cs = lam * torch.clamp(rhos, max=clip_c)
    vtp1 = torch.cat([values[1:], bootstrap[None]], 0)
    deltas = crho * (rewards + discounts * vtp1 - values)
    acc = torch.zeros_like(bootstrap)
    out = []
    for t in range(values.shape[0] - 1, -1, -1):
        acc = deltas[t] + discounts[t] * cs[t] * acc
        out.append(acc)
    vs_minus_v = torch.stack(out[::-1], 0)
    vs = values + vs_minus_v
    vs_tp1 = torch.cat([vs[1:], bootstrap[None]], 0)
    pg = torch.clamp(rhos, max=clip_pg_rho) * (rewards + discounts * vs_tp1 - values)
    return vs, pg


def ppo_loss(logits, old_logits, actions, old_logp, adv, vpred, vtarg, clip=0.2, vf_clip=10.0,
             vf_coeff=1.0, ent_coeff=0.0, kl_coeff=0.0):
    """RLlib PPO loss (ppo_torch_learner.compute_loss_for_module). Returns (total, stats)."""
    lp = torch.log_softmax(logits.float(), -1)
    logp = lp.gather(-1, actions.long()[:, None])[:, 0]
    ratio = torch.exp(logp - old_logp.float())
    surr = torch.minimum(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip))
    ent = -(lp.exp() * lp).sum(-1)
    if old_logits is not None:
        olp = torch.log_softmax(old_logits.float(), -1)
        kl = (olp.exp() * (olp - lp)).sum(-1)
    else:
        kl = torch.zeros_like(ent)
    if vpred is not None:
        vf = torch.clamp((vpred.float() - vtarg.float()) ** 2, 0, vf_clip)
    else:
        vf = torch.zeros_like(ent)
    total = (-surr + vf_coeff * vf - ent_coeff * ent + kl_coeff * kl).mean()
    clipfrac = ((ratio < 1 - clip) | (ratio > 1 + clip)).float().mean()
    stats = torch.stack([total.detach(), (-surr).mean().detach(), vf.mean().detach(),
                         ent.mean().detach(), kl.mean().detach(), clipfrac])
    return total, stats


def image_normalize(x_u8_nhwc, mean, std, out_dtype=torch.float32):
    x = x_u8_nhwc.float().div(255.0).permute(0, 3, 1, 2)
    m = torch.as_tensor(mean, dtype=torch.float32, device=x.device).view(1, -1, 1, 1)
    s = torch.as_tensor(std, dtype=torch.float32, device=x.device).view(1, -1, 1, 1)
    return ((x - m) / s).to(out_dtype).contiguous()
