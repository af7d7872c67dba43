"""Numerics of every HIP kernel vs a plain fp32 PyTorch reference (GPU only)."""

import pytest
import torch

from ray_amd.ops import _lib
from ray_amd.ops import functional as rf
from ray_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_lib(cuda_device):
    assert _lib.available(), "libray_amd_hip.so must load on a GPU box"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("N,D", [(1000, 768), (64, 1024), (33, 1600), (8, 256)])
def test_layernorm_fwd_bwd(cuda_device, N, D):
    torch.manual_seed(0)
    x = torch.randn(N, D, device=cuda_device).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(D, device=cuda_device)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(D, device=cuda_device)).bfloat16().requires_grad_()
    y = rf.layer_norm(x, w, b)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-5)
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2


@pytest.mark.parametrize("N,F", [(512, 3072), (37, 64), (4099, 3072)])
def test_bias_gelu(cuda_device, N, F):
    torch.manual_seed(1)
    h = torch.randn(N, F, device=cuda_device).bfloat16().requires_grad_()
    b = (0.5 * torch.randn(F, device=cuda_device)).bfloat16().requires_grad_()
    y = rf.bias_gelu(h, b)
    hr, br = h.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = ref.gelu_tanh(hr + br)
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert _rel(h.grad, hr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2


def test_bias_residual(cuda_device):
    torch.manual_seed(2)
    h = torch.randn(300, 768, device=cuda_device).bfloat16().requires_grad_()
    b = torch.randn(768, device=cuda_device).bfloat16().requires_grad_()
    r = torch.randn(300, 768, device=cuda_device).bfloat16().requires_grad_()
    y = rf.bias_residual(h, b, r)
    yr = h.detach().float() + b.detach().float() + r.detach().float()
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    assert _rel(b.grad, g.sum(0)) < 2e-2
    assert _rel(h.grad, g) < 1e-2


@pytest.mark.parametrize("N,V,Vp", [(256, 50257, 50304), (100, 1000, 1000)])
def test_cross_entropy(cuda_device, N, V, Vp):
    torch.manual_seed(3)
    logits = (3 * torch.randn(N, Vp, device=cuda_device)).bfloat16().requires_grad_()
    t = torch.randint(0, V, (N,), device=cuda_device)
    t[::17] = -100
    loss = rf.cross_entropy(logits, t, V)
    lr_ = logits.detach().float().requires_grad_()
    lref = torch.nn.functional.cross_entropy(lr_[:, :V], t, ignore_index=-100)
    assert abs(loss.item() - lref.item()) < 2e-3 * max(1.0, abs(lref.item()))
    loss.backward()
    lref.backward()
    assert _rel(logits.grad, lr_.grad) < 2e-2
    if Vp > V:
        assert logits.grad[:, V:].abs().max().item() == 0


@pytest.mark.parametrize("T,B", [(128, 8), (512, 16), (33, 2048), (1000, 3)])
def test_gae(cuda_device, T, B):
    torch.manual_seed(4)
    r = torch.randn(T, B, device=cuda_device)
    v = torch.randn(T, B, device=cuda_device)
    d = (torch.rand(T, B, device=cuda_device) < 0.05).float()
    bs = torch.randn(B, device=cuda_device)
    adv, vt = rf.gae(r, v, d, bs, 0.99, 0.95)
    adv_r, vt_r = ref.gae(r.double(), v.double(), d.double(), bs.double(), 0.99, 0.95)
    assert torch.allclose(adv.double(), adv_r.double(), atol=1e-3, rtol=1e-3)
    assert torch.allclose(vt.double(), vt_r.double(), atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("T,B", [(80, 32), (20, 4096), (300, 5)])
def test_vtrace(cuda_device, T, B):
    torch.manual_seed(5)
    lr_ = 0.5 * torch.randn(T, B, device=cuda_device)
    disc = 0.99 * (torch.rand(T, B, device=cuda_device) > 0.05).float()
    r = torch.randn(T, B, device=cuda_device)
    v = torch.randn(T, B, device=cuda_device)
    bs = torch.randn(B, device=cuda_device)
    vs, pg = rf.vtrace(lr_, disc, r, v, bs)
    vs_r, pg_r = ref.vtrace(lr_.double(), disc.double(), r.double(), v.double(), bs.double())
    assert torch.allclose(vs.double(), vs_r, atol=1e-3, rtol=1e-3)
    assert torch.allclose(pg.double(), pg_r, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("A", [2, 6, 18])
def test_ppo_loss(cuda_device, A):
    torch.manual_seed(6)
    N = 1000
    logits = torch.randn(N, A, device=cuda_device, requires_grad=True)
    old = (logits.detach() + 0.3 * torch.randn(N, A, device=cuda_device))
    acts = torch.randint(0, A, (N,), device=cuda_device)
    old_lp = torch.log_softmax(old, -1).gather(-1, acts[:, None])[:, 0]
    adv = torch.randn(N, device=cuda_device)
    vp = torch.randn(N, device=cuda_device, requires_grad=True)
    vt = torch.randn(N, device=cuda_device) * 3
    kw = dict(clip=0.2, vf_clip=4.0, vf_coeff=0.5, ent_coeff=0.01, kl_coeff=0.2)
    loss, stats = rf.ppo_loss(logits, old, acts, old_lp, adv, vp, vt, **kw)
    lr_ = logits.detach().clone().requires_grad_()
    vr = vp.detach().clone().requires_grad_()
    lref, sref = ref.ppo_loss(lr_, old, acts, old_lp, adv, vr, vt, **kw)
    assert abs(loss.item() - lref.item()) < 1e-4 * max(1, abs(lref.item()))
    assert torch.allclose(stats, sref, atol=1e-4, rtol=1e-3)
    loss.backward()
    lref.backward()
    assert torch.allclose(logits.grad, lr_.grad, atol=1e-6, rtol=1e-3)
    assert torch.allclose(vp.grad, vr.grad, atol=1e-6, rtol=1e-3)


def _ppo_case(dev, N, A, seed):
    torch.manual_seed(seed)
    logits = torch.randn(N, A, device=dev)
    old = logits + 0.3 * torch.randn(N, A, device=dev)
    acts = torch.randint(0, A, (N,), device=dev)
    old_lp = torch.log_softmax(old, -1).gather(-1, acts[:, None])[:, 0]
    adv = torch.randn(N, device=dev)
    vp = torch.randn(N, device=dev)
    vt = torch.randn(N, device=dev) * 3
    return logits, old, acts, old_lp, adv, vp, vt


def test_ppo_loss_bf16_heads(cuda_device):
    """bf16 logits / values are read directly by the kernel; grads come back bf16."""
    logits, old, acts, old_lp, adv, vp, vt = _ppo_case(cuda_device, 700, 6, 16)
    kw = dict(clip=0.2, vf_clip=4.0, vf_coeff=0.5, ent_coeff=0.01, kl_coeff=0.2)
    lb = logits.bfloat16().requires_grad_()
    vb = vp.bfloat16().requires_grad_()
    loss, stats = rf.ppo_loss(lb, old, acts, old_lp, adv, vb, vt, **kw)
    lr_ = lb.detach().float().requires_grad_()
    vr = vb.detach().float().requires_grad_()
    lref, sref = ref.ppo_loss(lr_, old, acts, old_lp, adv, vr, vt, **kw)
    assert torch.allclose(stats, sref, atol=1e-4, rtol=1e-3)
    (2.0 * loss).backward()
    (2.0 * lref).backward()
    assert lb.grad.dtype == torch.bfloat16 and vb.grad.dtype == torch.bfloat16
    assert _rel(lb.grad, lr_.grad) < 1e-2
    assert _rel(vb.grad, vr.grad) < 1e-2


def test_ppo_loss_packed_gathers_rows(cuda_device):
    """Packed behaviour table + in-kernel gather == loss over the gathered minibatch;
    stats accumulate across calls."""
    Nf, A, mb = 2000, 6, 500
    logits_f, old, acts, old_lp, adv, vp_f, vt = _ppo_case(cuda_device, Nf, A, 17)
    aux = rf.ppo_pack(old, acts, old_lp, adv, vt)
    idx = torch.randperm(Nf, device=cuda_device)[:mb]
    kw = dict(clip=0.2, vf_clip=4.0, vf_coeff=0.5, ent_coeff=0.01, kl_coeff=0.2)
    lg = logits_f[idx].bfloat16().requires_grad_()
    vv = vp_f[idx].bfloat16().requires_grad_()
    stats = torch.zeros(6, device=cuda_device)
    h = rf.ppo_loss_packed(lg, vv, aux, idx, stats, **kw)
    rf.ppo_loss_packed(lg.detach(), vv.detach(), aux, idx, stats, **kw)  # accumulates
    lr_ = lg.detach().float().requires_grad_()
    vr = vv.detach().float().requires_grad_()
    lref, sref = ref.ppo_loss(lr_, old[idx], acts[idx], old_lp[idx], adv[idx], vr, vt[idx], **kw)
    assert torch.allclose(stats, 2 * sref, atol=2e-4, rtol=1e-3)
    torch.autograd.backward(h, torch.ones((), device=cuda_device))
    lref.backward()
    assert _rel(lg.grad, lr_.grad) < 1e-2
    assert _rel(vv.grad, vr.grad) < 1e-2


@pytest.mark.parametrize("A,F", [(6, 512), (4, 256), (18, 1024)])
def test_ppo_heads_loss_matches_unfused(cuda_device, A, F):
    """Fused heads + PPO loss == bf16 linear heads followed by the packed loss kernel."""
    torch.manual_seed(23)
    Nf, mb = 900, 300
    h = torch.relu(torch.randn(mb, F, device=cuda_device)).bfloat16().requires_grad_()
    wpi = (0.05 * torch.randn(A, F, device=cuda_device)).bfloat16().requires_grad_()
    bpi = (0.1 * torch.randn(A, device=cuda_device)).bfloat16().requires_grad_()
    wvf = (0.05 * torch.randn(1, F, device=cuda_device)).bfloat16().requires_grad_()
    bvf = (0.1 * torch.randn(1, device=cuda_device)).bfloat16().requires_grad_()
    _, old, acts, old_lp, adv, _, vt = _ppo_case(cuda_device, Nf, A, 24)
    aux = rf.ppo_pack(old, acts, old_lp, adv, vt)
    idx = torch.randperm(Nf, device=cuda_device)[:mb]
    kw = dict(clip=0.2, vf_clip=4.0, vf_coeff=0.5, ent_coeff=0.01, kl_coeff=0.2)
    st = torch.zeros(6, device=cuda_device)
    hdl = rf.ppo_heads_loss(h, wpi, bpi, wvf, bvf, aux, idx, st, **kw)
    torch.autograd.backward(hdl, torch.full((), 2.0, device=cuda_device))
    refs = [t.detach().clone().requires_grad_() for t in (h, wpi, bpi, wvf, bvf)]
    lg = torch.nn.functional.linear(refs[0], refs[1], refs[2])
    v = torch.nn.functional.linear(refs[0], refs[3], refs[4]).squeeze(-1)
    st_r = torch.zeros(6, device=cuda_device)
    hr = rf.ppo_loss_packed(lg, v, aux, idx, st_r, **kw)
    torch.autograd.backward(hr, torch.full((), 2.0, device=cuda_device))
    assert torch.allclose(st, st_r, atol=2e-3, rtol=2e-2)
    for a_, b_ in zip((h, wpi, bpi, wvf, bvf), refs):
        assert _rel(a_.grad, b_.grad) < 2e-2


@pytest.mark.parametrize("shape", [(64, 32, 20, 20), (37, 64, 9, 9), (500, 64, 7, 7), (300, 512)])
def test_bias_relu(cuda_device, shape):
    torch.manual_seed(18)
    h = torch.randn(*shape, device=cuda_device).bfloat16()
    if h.dim() == 4:
        h = h.contiguous(memory_format=torch.channels_last)
    h.requires_grad_()
    C = shape[1]
    b = (0.3 * torch.randn(C, device=cuda_device)).bfloat16().requires_grad_()
    y = rf.bias_relu(h, b)
    assert y.shape == h.shape and y.stride() == h.stride()
    hr, br = h.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = torch.relu(hr + (br.view(1, -1, 1, 1) if h.dim() == 4 else br))
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    if h.dim() == 4:
        g = g.contiguous(memory_format=torch.channels_last)
    y.backward(g.bfloat16())
    yr.backward(g)
    # the mask comes from the bf16 output: rows where h+b rounds to exactly 0 may differ
    assert _rel(h.grad, hr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2


def test_linear_relu(cuda_device):
    torch.manual_seed(25)
    x = torch.randn(300, 3136, device=cuda_device).bfloat16().requires_grad_()
    w = (0.02 * torch.randn(512, 3136, device=cuda_device)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(512, device=cuda_device)).bfloat16().requires_grad_()
    y = rf.linear_relu(x, w, b)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.relu(torch.nn.functional.linear(xr, wr, br))
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    for a_, b_ in ((x, xr), (w, wr), (b, br)):
        assert _rel(a_.grad, b_.grad) < 2e-2


def test_bias_relu_flat_sink(cuda_device):
    """With a flat-managed bias the gradient is written into the flat buffer directly."""
    from ray_amd.parallel.flat import FlatParams

    torch.manual_seed(19)
    conv = torch.nn.Conv2d(4, 32, 8, 4).to(cuda_device).to(memory_format=torch.channels_last)
    flat = FlatParams(conv, dtype=torch.bfloat16, grad_dtype=torch.bfloat16)
    assert conv.weight.is_contiguous(memory_format=torch.channels_last)
    x = torch.randn(16, 84, 84, 4, device=cuda_device).bfloat16().permute(0, 3, 1, 2)
    flat.zero_grad()
    y = rf.bias_relu(torch.nn.functional.conv2d(x, conv.weight, None, 4), conv.bias)
    y.float().sum().backward()
    wr = conv.weight.detach().float().requires_grad_()
    br = conv.bias.detach().float().requires_grad_()
    yr = torch.relu(torch.nn.functional.conv2d(x.float(), wr, br, 4))
    yr.sum().backward()
    assert _rel(conv.bias._ra_grad, br.grad) < 2e-2
    assert _rel(conv.weight._ra_grad, wr.grad) < 2e-2


@pytest.mark.parametrize("cfg", [(84, 4, 32, 8, 4, True), (84, 4, 32, 8, 4, False),
                                 (20, 32, 64, 4, 2, False), (9, 64, 64, 3, 1, False)])
def test_conv_bias_relu(cuda_device, cfg):
    """MFMA NHWC conv (+bias+ReLU) fwd, weight grad (and MIOpen input grad) vs fp32 torch;
    the uint8 first layer gathers its rows by index."""
    HW, C, O, Kk, S, u8 = cfg
    torch.manual_seed(20)
    Nfull, B = 70, 45
    w = (torch.randn(O, C, Kk, Kk, device=cuda_device) / (C * Kk * Kk) ** 0.5).bfloat16()
    w = w.contiguous(memory_format=torch.channels_last).requires_grad_()
    b = (0.1 * torch.randn(O, device=cuda_device)).bfloat16().requires_grad_()
    idx = None
    if u8:
        frames = torch.randint(0, 256, (Nfull, HW, HW, C), dtype=torch.uint8, device=cuda_device)
        idx = torch.randperm(Nfull, device=cuda_device)[:B]
        x = frames
        xr = (frames[idx].float() * (1.0 / 255.0)).permute(0, 3, 1, 2)
    else:
        x0 = torch.randn(B, HW, HW, C, device=cuda_device).bfloat16().requires_grad_()
        x = x0.permute(0, 3, 1, 2)
        xr0 = x0.detach().float().requires_grad_()
        xr = xr0.permute(0, 3, 1, 2)
    y = rf.conv2d_bias_relu(x, w, b, S, idx=idx)
    wr = w.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_()
    yr = torch.relu(torch.nn.functional.conv2d(xr, wr, br, S))
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr).contiguous(memory_format=torch.channels_last)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert _rel(w.grad, wr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2
    if not u8:
        assert _rel(x0.grad, xr0.grad) < 2e-2


@pytest.mark.parametrize("u8", [True, False])
def test_conv_bias_relu_graph_replay(cuda_device, u8):
    """Captured in a HIP graph, the conv fwd + weight-grad kernels recompute on replay
    (new input values, same buffers) exactly like eager calls."""
    torch.manual_seed(22)
    if u8:
        HW, C, O, Kk, S = 84, 4, 32, 8, 4
        src = torch.randint(0, 256, (50, HW, HW, C), dtype=torch.uint8, device=cuda_device)
        idx = torch.randperm(50, device=cuda_device)[:32]
    else:
        HW, C, O, Kk, S = 9, 64, 64, 3, 1
        src = torch.randn(32, HW, HW, C, device=cuda_device).bfloat16()
        idx = None
    w = (torch.randn(O, C, Kk, Kk, device=cuda_device) * 0.05).bfloat16()
    w = w.contiguous(memory_format=torch.channels_last).requires_grad_()
    b = (0.1 * torch.randn(O, device=cuda_device)).bfloat16().requires_grad_()
    gy = torch.randn(32, (HW - Kk) // S + 1, (HW - Kk) // S + 1, O,
                     device=cuda_device).bfloat16().permute(0, 3, 1, 2)

    def step():
        x = src if u8 else src.permute(0, 3, 1, 2)
        y = rf.conv2d_bias_relu(x, w, b, S, idx=idx)
        gw, gb = torch.autograd.grad(y, (w, b), gy)
        return y, gw, gb

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = step()
    for _ in range(2):  # new values in the same buffers, then replay
        if u8:
            src.copy_(torch.randint(0, 256, src.shape, dtype=torch.uint8, device=cuda_device))
        else:
            src.copy_(torch.randn(src.shape, device=cuda_device).bfloat16())
        g.replay()
        ref_out = step()
        torch.cuda.synchronize()
        for a_, b_ in zip(out, ref_out):
            assert torch.equal(a_, b_)


def test_nature_cnn_fused_matches_eager(cuda_device):
    """The fused GPU encoder (u8 frames + idx) == the generic path on the same weights."""
    from ray_amd.rllib.core.rl_module import NatureCNN

    torch.manual_seed(21)
    net = NatureCNN((84, 84, 4)).to(cuda_device).bfloat16()
    net = net.to(memory_format=torch.channels_last)
    frames = torch.randint(0, 256, (64, 84, 84, 4), dtype=torch.uint8, device=cuda_device)
    idx = torch.randperm(64, device=cuda_device)[:40]
    h = net(frames, idx)
    ref_net = NatureCNN((84, 84, 4)).to(cuda_device)
    ref_net.load_state_dict({k: v.float() for k, v in net.state_dict().items()})
    hr = ref_net(frames[idx].float() * (1.0 / 255.0))
    assert _rel(h, hr) < 2e-2


def test_gather_cast_u8(cuda_device):
    x = torch.randint(0, 256, (300, 84, 84, 4), dtype=torch.uint8, device=cuda_device)
    idx = torch.randperm(300, device=cuda_device)[:77]
    y = rf.gather_cast_u8(x, idx)
    assert y.dtype == torch.bfloat16 and y.shape == (77, 84, 84, 4)
    yr = (x[idx].float() * (1.0 / 255.0)).bfloat16()
    assert torch.allclose(y.float(), yr.float(), atol=4e-3, rtol=0)


def test_obsnorm(cuda_device):
    torch.manual_seed(7)
    rms = rf.RunningMeanStd(17, device=cuda_device)
    cpu = rf.RunningMeanStd(17, device="cpu")
    for n in (5, 300, 1000):
        x = torch.randn(n, 17) * 3 + 2
        rms.update(x.to(cuda_device))
        cpu.update(x)
    assert torch.allclose(rms.mean.cpu(), cpu.mean, atol=1e-4)
    assert torch.allclose(rms.var.cpu(), cpu.var, atol=1e-3, rtol=1e-3)
    x = torch.randn(64, 17) * 3 + 2
    assert torch.allclose(rms.normalize(x.to(cuda_device)).cpu(), cpu.normalize(x), atol=1e-3)


def test_image_normalize(cuda_device):
    x = torch.randint(0, 256, (4, 37, 130, 3), dtype=torch.uint8, device=cuda_device)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    y = rf.image_normalize(x, mean, std)
    yr = ref.image_normalize(x.cpu(), mean, std)
    assert torch.allclose(y.cpu(), yr, atol=1e-5)
    yb = rf.image_normalize(x, mean, std, torch.bfloat16)
    assert _rel(yb, yr.to(cuda_device)) < 1e-2
    z = rf.resize_bilinear(y, (20, 64))
    zr = torch.nn.functional.interpolate(y, size=(20, 64), mode="bilinear", align_corners=False)
    assert torch.allclose(z, zr, atol=1e-4)
    c = rf.cast_scale_u8(x)
    assert _rel(c, x.float() / 255) < 1e-2


@pytest.mark.parametrize("C", [1, 3, 4])
def test_image_normalize_vector_path(cuda_device, C):
    """H*W % 16 == 0: the 16-pixels-per-thread kernel (16-byte loads/stores)."""
    x = torch.randint(0, 256, (5, 224, 224, C), dtype=torch.uint8, device=cuda_device)
    mean, std = [0.485, 0.456, 0.406, 0.5][:C], [0.229, 0.224, 0.225, 0.25][:C]
    yr = ref.image_normalize(x.cpu(), mean, std)
    y = rf.image_normalize(x, mean, std)
    assert y.shape == (5, C, 224, 224)
    assert torch.allclose(y.cpu(), yr, atol=1e-5)
    yb = rf.image_normalize(x, mean, std, torch.bfloat16)
    assert torch.allclose(yb.float().cpu(), yr, atol=2e-2, rtol=8e-3)


@pytest.mark.parametrize("B,T,H", [(2, 256, 3), (1, 1024, 2), (2, 128, 1)])
def test_flash_attention_fwd_bwd(cuda_device, B, T, H):
    """Causal attention forward, then dQ (computing delta) and dK/dV, against fp32
    autograd."""
    torch.manual_seed(9)
    D = 64
    qkv = torch.randn(B, T, 3, H, D, device=cuda_device).bfloat16().requires_grad_()
    y = rf.causal_attention_qkv(qkv)
    ref_in = qkv.detach().float().requires_grad_()
    q, k, v = ref_in.permute(2, 0, 3, 1, 4).unbind(0)
    s = (q @ k.transpose(-1, -2)) * D ** -0.5
    mask = torch.ones(T, T, device=cuda_device, dtype=torch.bool).triu(1)
    p = torch.softmax(s.masked_fill(mask, float("-inf")), -1)
    yr = (p @ v).transpose(1, 2)
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert _rel(qkv.grad, ref_in.grad) < 2e-2
    for i in range(3):
        assert _rel(qkv.grad[:, :, i], ref_in.grad[:, :, i]) < 2e-2, i


@pytest.mark.parametrize("spike", [6.0, 20.0, 80.0])
def test_flash_attention_lazy_rescale_forced(cuda_device, spike):
    """The forward keeps a stale running max until a tile max exceeds it by > 8 (log2
    units). Spiking key rows at later tiles (aligned with every query) forces the rescale
    branch mid-sequence, at several spike sizes around the threshold; full fp32 reference
    (guide rule 26: a rare data-dependent branch needs an input that takes it)."""
    torch.manual_seed(19)
    B, T, H, D = 2, 512, 2, 64
    qkv = torch.randn(B, T, 3, H, D, device=cuda_device) * 0.5
    q_dir = torch.randn(D, device=cuda_device)
    q_dir /= q_dir.norm()
    qkv[:, :, 0] += q_dir * 2.0  # every query has a component along q_dir
    for t in (130, 300, 450):  # keys in later tiles that jump the row max
        qkv[:, t, 1] += q_dir * spike * (t / 150)
    qkv = qkv.bfloat16().requires_grad_()
    y = rf.causal_attention_qkv(qkv)
    ref_in = qkv.detach().double().requires_grad_()
    q, k, v = ref_in.permute(2, 0, 3, 1, 4).unbind(0)
    s = (q @ k.transpose(-1, -2)) * D ** -0.5
    mask = torch.ones(T, T, device=cuda_device, dtype=torch.bool).triu(1)
    p = torch.softmax(s.masked_fill(mask, float("-inf")), -1)
    yr = (p @ v).transpose(1, 2)
    assert torch.isfinite(y.float()).all()
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert _rel(qkv.grad, ref_in.grad) < 2e-2


def test_flat_adamw_matches_torch(cuda_device):
    from ray_amd.parallel.flat import FlatAdamW, FlatParams

    torch.manual_seed(8)
    m1 = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.LayerNorm(128),
                             torch.nn.Linear(128, 8)).to(cuda_device)
    m2 = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.LayerNorm(128),
                             torch.nn.Linear(128, 8)).to(cuda_device)
    m2.load_state_dict(m1.state_dict())
    flat = FlatParams(m1, dtype=torch.float32)
    opt = FlatAdamW(flat, lr=1e-2, weight_decay=0.1, max_grad_norm=None)
    decay = [p for p in m2.parameters() if p.dim() >= 2]
    nod = [p for p in m2.parameters() if p.dim() < 2]
    topt = torch.optim.AdamW([{"params": decay, "weight_decay": 0.1},
                              {"params": nod, "weight_decay": 0.0}], lr=1e-2, betas=(0.9, 0.95),
                             eps=1e-8)
    for _ in range(5):
        x = torch.randn(32, 64, device=cuda_device)
        flat.zero_grad()
        m1(x).square().mean().backward()
        opt.step()
        topt.zero_grad()
        m2(x).square().mean().backward()
        topt.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(a, b, atol=1e-5, rtol=1e-4)


def test_gpt2_tiny_trains(cuda_device):
    from ray_amd.models.gpt2 import GPT2Config
    from ray_amd.train.gpt2_step import GPT2Trainer

    cfg = GPT2Config.tiny()
    tr = GPT2Trainer(cfg, 8, 64, cuda_device, lr=3e-3, warmup_steps=2, total_steps=60)
    x, y = tr.synthetic_batch()
    first = None
    for _ in range(40):
        loss = float(tr.step([(x, y)]))
        first = first or loss
    assert loss < first * 0.7, (first, loss)


@pytest.mark.parametrize("M,N,K,bias", [(16384, 256, 256, True), (1000, 384, 128, False),
                                        (65536, 256, 256, False)])
def test_linear_splitk(cuda_device, M, N, K, bias):
    torch.manual_seed(10)
    x = torch.randn(M, K, device=cuda_device).bfloat16().requires_grad_()
    w = (0.05 * torch.randn(N, K, device=cuda_device)).bfloat16().requires_grad_()
    b = torch.randn(N, device=cuda_device).bfloat16().requires_grad_() if bias else None
    y = rf.linear(x, w, b)
    xr, wr = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_() if bias else None
    yr = torch.nn.functional.linear(xr, wr, br)
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 1e-2
    if bias:
        assert _rel(b.grad, br.grad) < 1e-2


def test_layer_norm_fork(cuda_device):
    torch.manual_seed(11)
    x = torch.randn(512, 768, device=cuda_device).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(768, device=cuda_device)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(768, device=cuda_device)).bfloat16().requires_grad_()
    skip, y = rf.layer_norm_fork(x, w, b)
    out = skip * 0.5 + y
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    outr = xr * 0.5 + torch.nn.functional.layer_norm(xr, (768,), wr, br, 1e-5)
    g = torch.randn_like(outr)
    out.backward(g.bfloat16())
    outr.backward(g)
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2 and _rel(b.grad, br.grad) < 2e-2


def test_flat_direct_grads_match_autograd(cuda_device):
    """GPT-2 tiny: grads accumulated in place into the flat buffer (sinks, split-K, LN fork)
    equal the plain autograd grads, and every DDP bucket is signalled exactly once."""
    import copy
    import os

    import torch.distributed as dist

    from ray_amd.models.gpt2 import GPT2, GPT2Config
    from ray_amd.parallel.flat import FlatDDP, FlatParams

    torch.manual_seed(12)
    cfg = GPT2Config(vocab_size=512, padded_vocab=512, n_positions=256, n_embd=128, n_layer=2,
                     n_head=2)
    a = GPT2(cfg).to(cuda_device).bfloat16()
    b = copy.deepcopy(a)
    idx = torch.randint(0, 512, (8, 256), device=cuda_device)
    tgt = torch.randint(0, 512, (8, 256), device=cuda_device)
    a(idx, tgt).backward()
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1)
    flat = FlatParams(b)
    ddp = FlatDDP(flat, bucket_mb=0.05, always_hook=True)
    assert len(ddp.buckets) > 2
    b(idx, tgt).backward()
    assert ddp._ready == ddp.bucket_sizes  # each param signalled once
    ddp.finish()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert _rel(pb._ra_grad, pa.grad) < 3e-2, n


def test_residual_layer_norm(cuda_device):
    torch.manual_seed(13)
    N, D = 2048, 768
    h = torch.randn(N, D, device=cuda_device).bfloat16().requires_grad_()
    skip = torch.randn(N, D, device=cuda_device).bfloat16().requires_grad_()
    rb = (0.1 * torch.randn(D, device=cuda_device)).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(D, device=cuda_device)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(D, device=cuda_device)).bfloat16().requires_grad_()
    x, y = rf.residual_layer_norm(h, rb, skip, w, b)
    hr, sr, rbr, wr, br = (t.detach().float().requires_grad_() for t in (h, skip, rb, w, b))
    xr = hr + rbr + sr
    yr = torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-5)
    assert _rel(x, xr) < 1e-2 and _rel(y, yr) < 1e-2
    gx, gy = torch.randn_like(xr), torch.randn_like(yr)
    torch.autograd.backward([x, y], [gx.bfloat16(), gy.bfloat16()])
    torch.autograd.backward([xr, yr], [gx, gy])
    for a, r in ((h, hr), (skip, sr), (rb, rbr), (w, wr), (b, br)):
        assert _rel(a.grad, r.grad) < 2e-2


@pytest.mark.parametrize("M,N,K", [(8192, 768, 768), (8192, 2304, 768), (4096, 3072, 768),
                                   (4096, 768, 3072), (2048, 50304, 768)])
def test_lt_wgrad_accum_matches_fp32(cuda_device, M, N, K):
    """hipBLASLt fp32-output selector: out = dy^T x + out, beta 0 and 1, tuned and default."""
    from ray_amd.ops import lt

    g = torch.Generator(device=cuda_device).manual_seed(0)
    dy = torch.randn(M, N, device=cuda_device, generator=g).to(torch.bfloat16)
    x = torch.randn(M, K, device=cuda_device, generator=g).to(torch.bfloat16)
    ref_ = dy.float().t() @ x.float()
    out = torch.full((N, K), 7.0, device=cuda_device)
    lt.wgrad_accum(dy, x, out, beta=0.0)
    assert _rel(out, ref_) < 1e-5
    lt.wgrad_accum(dy, x, out, beta=1.0)
    assert _rel(out, 2 * ref_) < 1e-5
    lt.set_tuning(True)
    try:
        lt._applied.clear()
        out2 = torch.zeros((N, K), device=cuda_device)
        lt.wgrad_accum(dy, x, out2)
        assert _rel(out2, ref_) < 1e-5
    finally:
        lt.set_tuning(False)


def test_lt_wgrad_partials_match_fp32(cuda_device):
    from ray_amd.ops import lt

    g = torch.Generator(device=cuda_device).manual_seed(1)
    dy = torch.randn(16384, 768, device=cuda_device, generator=g).to(torch.bfloat16)
    x = torch.randn(16384, 2304, device=cuda_device, generator=g).to(torch.bfloat16)
    part = lt.wgrad_partials(dy, x, 8)
    assert part.shape == (8, 768, 2304)
    ref_ = dy.float().view(8, 2048, 768).transpose(1, 2) @ x.float().view(8, 2048, 2304)
    assert _rel(part, ref_) < 1e-5


# ------------------------------------------------------------ hand-written MFMA GEMM
@pytest.mark.parametrize("M,N,K", [(512, 768, 256), (300, 196, 128), (1024, 788, 64),
                                   (256, 260, 3072)])
def test_gemm_nt_matches_fp32(cuda_device, M, N, K):
    """ops/csrc/gemm.hip against an fp32 torch reference, including
    ragged M / N edges (clamped loads, masked stores) and asymmetric operands."""
    from ray_amd.ops import gemm

    g = torch.Generator(device=cuda_device).manual_seed(M + N + K)
    a = torch.randn(M, K, device=cuda_device, generator=g).to(torch.bfloat16)
    b = (torch.randn(N, K, device=cuda_device, generator=g) * 0.1).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda_device, generator=g).to(torch.bfloat16)
    ref_c = a.float() @ b.float().t()
    out = gemm.gemm_nt(a, b)
    torch.testing.assert_close(out.float(), ref_c, rtol=2e-2, atol=2e-2 * ref_c.abs().max().item())
    out_b = gemm.gemm_nt(a, b, epi="bias", bias=bias)
    torch.testing.assert_close(out_b.float(), ref_c + bias.float(), rtol=2e-2,
                               atol=2e-2 * ref_c.abs().max().item())
    y, pre = gemm.gemm_nt(a, b, epi="bias_gelu", bias=bias)
    torch.testing.assert_close(pre.float(), ref_c, rtol=2e-2,
                               atol=2e-2 * ref_c.abs().max().item())
    y_ref = torch.nn.functional.gelu(pre.float() + bias.float(), approximate="tanh")
    torch.testing.assert_close(y.float(), y_ref, rtol=2e-2, atol=2e-2 * y_ref.abs().max().item())
    # GELU backward + bias gradient: dh = (dy @ w2t^T) * gelu'(pre + bias), db += sum(dh)
    dy = torch.randn(M, K, device=cuda_device, generator=g).to(torch.bfloat16)
    w2t = b  # [N, K]
    db = torch.full((N,), 0.5, device=cuda_device)
    dh = gemm.gemm_nt(dy, w2t, epi="dgelu", bias=bias, aux=pre, db=db, db_acc=True)
    u = (pre.float() + bias.float()).requires_grad_(True)
    gd = torch.autograd.grad(torch.nn.functional.gelu(u, approximate="tanh"), u,
                             dy.float() @ w2t.float().t())[0]
    torch.testing.assert_close(dh.float(), gd, rtol=2e-2, atol=2e-2 * gd.abs().max().item())
    torch.testing.assert_close(db, 0.5 + gd.sum(0), rtol=2e-2,
                               atol=2e-2 * gd.sum(0).abs().max().item())


@pytest.mark.parametrize("N,D,res", [(5003, 768, True), (4099, 1024, False), (37, 256, True),
                                     (70000, 768, True)])
def test_layernorm_bwd_v2_matches_fp32(cuda_device, N, D, res):
    """Branch-free buffer-op LayerNorm backward (v2: D % 256 == 0): dx (+ skip gradient),
    dgamma, dbeta and the residual-bias colsum against fp32 autograd, with a row count
    that leaves the last row pair of some waves past N."""
    from ray_amd.ops import _lib

    torch.manual_seed(21)
    h = torch.randn(N, D, device=cuda_device).bfloat16().requires_grad_()
    skip = torch.randn(N, D, device=cuda_device).bfloat16().requires_grad_()
    rb = (0.1 * torch.randn(D, device=cuda_device)).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(D, device=cuda_device)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(D, device=cuda_device)).bfloat16().requires_grad_()
    hr, sr, rbr, wr, br = (t.detach().float().requires_grad_() for t in (h, skip, rb, w, b))
    gy = torch.randn(N, D, device=cuda_device)
    gx = torch.randn(N, D, device=cuda_device)
    if res:
        x, y = rf.residual_layer_norm(h, rb, skip, w, b)
        torch.autograd.backward([x, y], [gx.bfloat16(), gy.bfloat16()])
        xr = hr + rbr + sr
        yr = torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-5)
        torch.autograd.backward([xr, yr], [gx, gy])
        pairs = ((h, hr), (skip, sr), (rb, rbr), (w, wr), (b, br))
    else:
        y = rf.layer_norm(h, w, b)
        y.backward(gy.bfloat16())
        yr = torch.nn.functional.layer_norm(hr, (D,), wr, br, 1e-5)
        yr.backward(gy)
        pairs = ((h, hr), (w, wr), (b, br))
    for a, r in pairs:
        assert _rel(a.grad, r.grad) < 2e-2


@pytest.mark.parametrize("N,D,res", [(5003, 768, True), (65536, 768, False)])
def test_layernorm_bwd_fp32_sinks_accumulate(cuda_device, N, D, res):
    """Flat-gradient contract of ra_layernorm_bwd (fp32 sinks, accumulate): dgamma, dbeta
    and the residual-bias colsum are ADDED onto non-zero sinks by in-kernel atomics."""
    from ray_amd.ops import _lib
    from ray_amd.ops._lib import check, ptr, stream_ptr

    L = _lib.lib()
    torch.manual_seed(5)
    x = torch.randn(N, D, device=cuda_device).bfloat16()
    w = (1 + 0.1 * torch.randn(D, device=cuda_device)).bfloat16()
    dy = torch.randn(N, D, device=cuda_device).bfloat16()
    dres = torch.randn(N, D, device=cuda_device).bfloat16() if res else None
    xf = x.float()
    mean = xf.mean(1)
    rstd = torch.rsqrt(xf.var(1, unbiased=False) + 1e-5)
    xh = (xf - mean[:, None]) * rstd[:, None]
    g = dy.float() * w.float()
    dxr = (g - g.mean(1, keepdim=True) - xh * (g * xh).mean(1, keepdim=True)) * rstd[:, None]
    if res:
        dxr = dxr + dres.float()
    init = [torch.randn(D, device=cuda_device) for _ in range(3)]
    sinks = [t.clone() for t in init]
    dx = torch.empty_like(x)
    work = torch.empty(L.ra_layernorm_bwd_work(N, D), device=cuda_device, dtype=torch.float32)
    check(L.ra_layernorm_bwd(ptr(dy), ptr(x), ptr(w), ptr(mean), ptr(rstd), ptr(dres),
                             ptr(dx), ptr(sinks[0]), ptr(sinks[1]),
                             ptr(sinks[2]) if res else None, ptr(work), N, D, 2,
                             stream_ptr()), "layernorm_bwd")
    torch.cuda.synchronize()
    assert _rel(dx, dxr) < 2e-2
    assert _rel(sinks[0] - init[0], (dy.float() * xh).sum(0)) < 1e-3
    assert _rel(sinks[1] - init[1], dy.float().sum(0)) < 1e-3
    if res:
        assert _rel(sinks[2] - init[2], dx.float().sum(0)) < 1e-2
    else:
        assert torch.equal(sinks[2], init[2])


@pytest.mark.parametrize("S", [1, 2, 3, 4, 8, 16])
@pytest.mark.parametrize("f32,acc", [(True, True), (True, False), (False, True)])
def test_splitk_accum_matches_fp32(cuda_device, S, f32, acc):
    """ra_splitk_accum: grad (+)= sum_s part[s] for the fixed-S kernels (S = 2..16) and the
    runtime-S fallback, fp32 and bf16 gradients."""
    from ray_amd.ops import _lib
    from ray_amd.ops._lib import ptr, stream_ptr

    torch.manual_seed(S)
    n = 4 * 12345
    part = torch.randn(S, n, device=cuda_device)
    g0 = torch.randn(n, device=cuda_device)
    grad = g0.clone() if f32 else g0.bfloat16()
    want = part.sum(0) + (grad.float() if acc else 0)
    rc = _lib.lib().ra_splitk_accum(ptr(part), S, n, ptr(grad), (1 if acc else 0) | (2 if f32 else 0),
                                    stream_ptr())
    assert rc == 0
    assert _rel(grad.float(), want) < (1e-6 if f32 else 5e-3)


@pytest.mark.parametrize("rows,cols", [(768, 2304), (3072, 768), (70, 130)])
def test_transpose_bf16_kernel(cuda_device, rows, cols):
    """LDS-tiled bf16 transpose (the transposed-weight copy) vs torch, ragged edges incl."""
    w = torch.randn(rows, cols, device=cuda_device).bfloat16()
    wt = torch.full((cols, rows), 7.0, device=cuda_device, dtype=torch.bfloat16)
    st = torch.cuda.current_stream(cuda_device).cuda_stream
    assert _lib.lib().ra_transpose_bf16(w.data_ptr(), wt.data_ptr(), rows, cols, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(wt, w.t())


# ----------------------------------------------------------------- hand-written wgrad kernel
@pytest.mark.parametrize("M,N,K,bias,sdtype", [
    (65536 // 16, 2304, 768, True, torch.float32),   # GPT-2 qkv shape, fewer tokens
    (4096, 768, 3072, False, torch.float32),          # mlp_proj
    (1000, 264, 136, True, torch.float32),            # ragged N, K (not multiples of 256), token tail
    (640, 72, 40, True, torch.bfloat16),              # bf16 sink, tiny ragged tiles
    (64 * 300, 3072, 3072, False, torch.float32),     # S == 1 path (144 tiles... or split)
])
def test_wgrad_kernel_matches_fp32(cuda_device, M, N, K, bias, sdtype):
    """ops/csrc/wgrad.hip vs an fp32 torch reference: dW += dY^T X, db += colsum(dY),
    accumulated onto a non-zero sink (the flat-gradient contract)."""
    torch.manual_seed(11)
    dy = torch.randn(M, N, device=cuda_device).bfloat16()
    x = torch.randn(M, K, device=cuda_device).bfloat16()
    sink0 = torch.randn(N, K, device=cuda_device)
    bsink0 = torch.randn(N, device=cuda_device)
    sink = sink0.to(sdtype).clone()
    bsink = bsink0.to(sdtype).clone() if bias else None
    assert rf._wgrad_hip_ok(dy, x, sink, bsink)
    rf.wgrad_accumulate(dy, x, sink, bsink)
    ref_w = sink0.to(sdtype).float() + dy.float().t() @ x.float()
    assert _rel(sink, ref_w) < (2e-3 if sdtype == torch.float32 else 1e-2)
    if bias:
        ref_b = bsink0.to(sdtype).float() + dy.float().sum(0)
        assert _rel(bsink, ref_b) < (2e-3 if sdtype == torch.float32 else 1e-2)
    # overwrite mode (accumulate=False)
    out = torch.full((N, K), 7.0, device=cuda_device)
    rf.wgrad_accumulate(dy, x, out, accumulate=False)
    assert _rel(out, dy.float().t() @ x.float()) < 2e-3


def test_wgrad_kernel_many_tiles_split(cuda_device):
    """More 256 x 256 tiles than CUs (the LM head's dW, vocab x C): ra_wgrad_splits picks
    the split count with the fewest partly-filled waves (3 at 591 tiles on 256 CUs) and the
    slab-summed result matches fp32, with the padded vocabulary rows exactly zero."""
    L = _lib.lib()
    cus = torch.cuda.get_device_properties(cuda_device).multi_processor_count
    if cus == 256:
        assert L.ra_wgrad_splits(65536, 50304, 768) == 3
    torch.manual_seed(14)
    M, V, Vp, C = 2048, 50257, 50304, 768
    lg = torch.randn(M, Vp, device=cuda_device).bfloat16()
    lg[:, V:] = 0
    h = torch.randn(M, C, device=cuda_device).bfloat16()
    dw = torch.full((Vp, C), 3.0, device=cuda_device)
    assert rf._wgrad_hip_ok(lg, h, dw)
    rf.wgrad_accumulate(lg, h, dw, accumulate=False)
    assert _rel(dw, lg.float().t() @ h.float()) < 2e-3
    assert float(dw[V:].abs().max()) == 0.0


def test_wgrad_kernel_strided_rows(cuda_device):
    """Operands that are column slices of wider rows (ld > N / K), as packed activations."""
    torch.manual_seed(12)
    big = torch.randn(2048, 1024, device=cuda_device).bfloat16()
    dy, x = big[:, :512], big[:, 512:768]
    sink = torch.zeros(512, 256, device=cuda_device)
    assert rf._wgrad_hip_ok(dy, x, sink)
    rf.wgrad_accumulate(dy, x, sink)
    assert _rel(sink, dy.float().t() @ x.float()) < 2e-3


def test_linear_hip_wgrad_fused_bias_into_flat_sinks(cuda_device, monkeypatch):
    """_Linear backward: weight and bias gradients land in the flat fp32 sinks from one
    kernel, matching autograd in fp32."""
    torch.manual_seed(13)
    M, K, N = 1024, 256, 768
    x = torch.randn(M, K, device=cuda_device).bfloat16().requires_grad_()
    w = (0.05 * torch.randn(N, K, device=cuda_device)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(N, device=cuda_device)).bfloat16().requires_grad_()
    flat = torch.zeros(N * K + N, device=cuda_device)
    w._ra_grad, w._ra_direct_grad = flat[:N * K].view(N, K), True
    b._ra_grad, b._ra_direct_grad = flat[N * K:], True
    y = rf.linear(x, w, b)
    g = torch.randn_like(y)
    y.backward(g)
    torch.cuda.synchronize()
    rf.join_side_streams()
    torch.cuda.synchronize()
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    torch.nn.functional.linear(xr, wr, br).backward(g.float())
    assert _rel(w._ra_grad, wr.grad) < 5e-3
    assert _rel(b._ra_grad, br.grad) < 5e-3
    assert _rel(x.grad, xr.grad) < 2e-2


def test_embedding_backward_into_flat_sinks(cuda_device):
    """ra_embed_bwd (ops/csrc/embed.hip): token-table scatter-add (duplicate ids included)
    and position batch-sum into pre-filled fp32 sinks vs the fp32 torch reference."""
    torch.manual_seed(15)
    B, T, C, V, P = 8, 96, 768, 1000, 128
    idx = torch.randint(0, 40, (B, T), device=cuda_device)  # many duplicates
    wte = torch.zeros(V, C, device=cuda_device).bfloat16()
    wpe = torch.zeros(P, C, device=cuda_device).bfloat16()
    flat = torch.randn(V * C + P * C, device=cuda_device)
    ref_flat = flat.clone()
    wte._ra_grad, wte._ra_direct_grad = flat[:V * C].view(V, C), True
    wpe._ra_grad, wpe._ra_direct_grad = flat[V * C:].view(P, C), True
    wte.requires_grad_()
    wpe.requires_grad_()
    x = rf.embedding(idx, wte, wpe)
    dx = torch.randn_like(x)
    x.backward(dx)
    torch.cuda.synchronize()
    d2 = dx.float().reshape(-1, C)
    ref_wte = ref_flat[:V * C].view(V, C).index_add(0, idx.reshape(-1), d2)
    ref_wpe = ref_flat[V * C:].view(P, C).clone()
    ref_wpe[:T] += dx.float().sum(0)
    assert _rel(wte._ra_grad, ref_wte) < 1e-5
    assert _rel(wpe._ra_grad, ref_wpe) < 1e-5
    assert wte.grad is None and wpe.grad is None
