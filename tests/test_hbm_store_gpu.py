"""HBM object store under pressure and across paths (GPU only): non-blocking sealed puts,
eviction + spill of a small arena to the host store, copy-on-get, the holder's peer-copy
path, and a Train worker consuming a GPU object another actor produced."""

import pytest
import torch

import ray_amd as ray
from ray_amd._private import gpu_object_store as gos

pytestmark = pytest.mark.gpu


@pytest.fixture
def small_arena(cuda_device, monkeypatch):
    monkeypatch.setattr(gos, "_DEFAULT_ARENA", 64 << 20)  # 64 MiB arena per GPU
    ray.init(num_cpus=4, num_gpus=1)
    yield
    ray.shutdown()


def test_put_is_sealed_asynchronously_and_readable(small_arena):
    t = torch.randn(1 << 20, device="cuda")
    r = ray.put(t)  # returns without synchronising the producer stream
    u = ray.get(r)
    assert torch.equal(u, t)
    gos.flush()
    assert gos.stats["puts"] >= 1


def test_arena_pressure_spills_to_host_and_restores(small_arena):
    ts = [torch.full((4 << 20,), float(i), device="cuda") for i in range(10)]  # 10 x 16 MiB
    refs = [ray.put(t) for t in ts]
    gos.flush()
    assert gos.stats["spilled"] > 0  # 160 MiB of primaries through a 64 MiB arena
    for i, r in enumerate(refs):
        v = ray.get(r)
        assert v.is_cuda and float(v[0]) == float(i) and float(v[-1]) == float(i)
    del refs
    import gc

    gc.collect()


def test_copy_on_get_hands_out_private_copies(small_arena, monkeypatch):
    r = ray.put(torch.arange(1000, device="cuda", dtype=torch.float32))
    a = ray.get(r)
    monkeypatch.setattr(gos, "COPY_ON_GET", True)
    b = ray.get(r)
    c = ray.get(r)
    assert b.data_ptr() != c.data_ptr() and b.data_ptr() != a.data_ptr()
    b.add_(1)  # writing a private copy never changes the stored object
    assert torch.equal(ray.get(r), torch.arange(1000, device="cuda", dtype=torch.float32))


def test_holder_peer_copy_path(small_arena, monkeypatch):
    """The path a reader on another (non-addressable) GPU takes: the source arena's holder
    copies the sub-object into the reader GPU's arena. On a 1-GPU box source == dest."""
    r = ray.put(torch.arange(1 << 16, device="cuda", dtype=torch.int32))
    gos.flush()
    monkeypatch.setattr(gos, "FORCE_PEER", True)
    before = gos.stats["peer_copies"]
    v = ray.get(r)
    assert gos.stats["peer_copies"] == before + 1
    assert torch.equal(v.cpu(), torch.arange(1 << 16, dtype=torch.int32))
    v2 = ray.get(r)  # the secondary copy is reused, no second peer copy
    assert gos.stats["peer_copies"] == before + 1 and torch.equal(v2, v)


def test_train_worker_consumes_gpu_object_from_actor(small_arena):
    from ray_amd import train
    from ray_amd.train import RunConfig, ScalingConfig
    from ray_amd.train.torch import TorchTrainer

    @ray.remote(num_gpus=0.01)
    class Producer:
        def make(self):
            return torch.full((1 << 18,), 2.0, device="cuda", dtype=torch.bfloat16)

    p = Producer.remote()
    ref = p.make.remote()

    def loop(config):
        t = ray.get(config["refs"][0])
        train.report({"sum": float(t.float().sum()), "cuda": bool(t.is_cuda)})

    # fractional GPU per worker so producer and trainer share the single GPU
    res = TorchTrainer(loop, train_loop_config={"refs": [ref]},
                       scaling_config=ScalingConfig(num_workers=1, use_gpu=True,
                                                    resources_per_worker={"GPU": 0.5}),
                       run_config=RunConfig(storage_path="/tmp/ra_hbm_t")).fit()
    assert res.metrics["cuda"] and res.metrics["sum"] == 2.0 * (1 << 18)
