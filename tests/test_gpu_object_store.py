"""HBM object store: CUDA tensors put/get zero-copy across processes (GPU only)."""

import pytest
import torch

import ray_amd as ray

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_cluster(cuda_device):
    ray.init(num_cpus=4, num_gpus=1)
    yield
    ray.shutdown()


def test_put_get_cuda_tensor_same_process(gpu_cluster):
    t = torch.arange(1 << 20, dtype=torch.float32, device="cuda")
    r = ray.put(t)
    u = ray.get(r)
    assert u.is_cuda and torch.equal(u, t)
    assert u.data_ptr() != t.data_ptr()  # lives in the HBM arena


@ray.remote(num_gpus=0.25)
class GpuActor:
    def make(self, n):
        return torch.full((n,), 3.0, device="cuda", dtype=torch.bfloat16)

    def consume(self, t):
        return float(t.float().sum()), t.is_cuda, t.data_ptr()

    def get_sum(self, r):
        t = ray.get(r[0])
        return float(t.float().sum())


def test_cross_process_zero_copy(gpu_cluster):
    a = GpuActor.remote()
    b = GpuActor.remote()
    ref = a.make.remote(1 << 20)          # produced on GPU by actor a, returned via HBM store
    s, is_cuda, p1 = ray.get(b.consume.remote(ref))  # consumed by actor b without host copy
    assert is_cuda and s == 3.0 * (1 << 20)
    s2, _, p2 = ray.get(b.consume.remote(ref))
    assert p1 == p2  # same arena bytes, no copy on the second get either
    t = torch.ones(1000, device="cuda") * 2
    r = ray.put(t)
    assert ray.get(b.get_sum.remote([r])) == 2000.0
    local = ray.get(ref)
    assert local.is_cuda and float(local.float().sum()) == 3.0 * (1 << 20)
