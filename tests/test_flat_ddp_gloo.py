"""FlatDDP across two gloo ranks (CPU): every bucket's all-reduce is launched by the
readiness hooks WHILE backward runs (before finish()), buckets launch in the same order on
both ranks, and after finish() the flat gradient equals the mean of the ranks' local
gradients (reference: python/ray/train/torch/train_loop_utils.py prepare_model -> DDP)."""
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ray_amd.parallel.flat import FlatDDP, FlatParams


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.Tanh(),
                               torch.nn.Linear(256, 256), torch.nn.Tanh(),
                               torch.nn.Linear(256, 8))


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _model()
        flat = FlatParams(m, dtype=torch.float32, grad_dtype=torch.float32)
        ddp = FlatDDP(flat, bucket_mb=0.1)
        order = []
        orig = ddp._launch

        def spy(b):
            order.append(b)
            return orig(b)

        ddp._launch = spy
        g = torch.Generator().manual_seed(100 + rank)
        x = torch.randn(32, 64, generator=g)
        y = torch.randn(32, 8, generator=g)
        flat.zero_grad()
        loss = ((m(x) - y) ** 2).mean()
        loss.backward()
        launched_in_backward = ddp.launched
        ddp.finish()
        reduced = flat.g.clone() * ddp.grad_scale
        # reference: each rank's local gradient, averaged with an explicit all_reduce
        ref_m = _model()
        ((ref_m(x) - y) ** 2).mean().backward()
        local = torch.cat([p.grad.reshape(-1) for p in ref_m.parameters()])
        dist.all_reduce(local)
        local /= world
        # map flat offsets back to the reference parameter order by name
        by_name = dict(zip(flat.names, flat.offsets))
        got = torch.cat([reduced[by_name[n]:by_name[n] + p.numel()]
                         for n, p in ref_m.named_parameters()])
        out[rank] = {"launched_in_backward": launched_in_backward,
                     "buckets": len(ddp.buckets), "order": order,
                     "max_err": float((got - local).abs().max())}
    finally:
        dist.destroy_process_group()


def test_flat_ddp_buckets_overlap_backward_gloo():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    r0, r1 = out[0], out[1]
    assert r0["buckets"] > 1
    # every bucket went out from the hooks during backward, in the same order on both ranks
    assert r0["launched_in_backward"] == r0["buckets"] == r1["launched_in_backward"]
    assert r0["order"] == r1["order"] and sorted(r0["order"]) == list(range(r0["buckets"]))
    assert r0["max_err"] < 1e-5 and r1["max_err"] < 1e-5
