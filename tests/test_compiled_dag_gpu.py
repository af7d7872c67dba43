"""Compiled DAG moving CUDA tensors between actors through the HBM arena
(reference: python/ray/dag/tests/experimental/test_torch_tensor_dag.py)."""

import pytest
import torch

import ray_amd as ray
from ray_amd.dag import InputNode

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4, num_gpus=1)
    yield
    ray.shutdown()


@ray.remote(num_gpus=0.5)
class Producer:
    def make(self, n):
        return torch.full((n, 1024), float(n), device="cuda", dtype=torch.bfloat16)


@ray.remote(num_gpus=0.5)
class Consumer:
    def reduce(self, t):
        assert t.is_cuda
        return float(t.float().sum().item())


def test_gpu_tensor_pipeline(cluster):
    p, c = Producer.remote(), Consumer.remote()
    with InputNode() as inp:
        dag = c.reduce.bind(p.make.bind(inp).with_tensor_transport())
    cdag = dag.experimental_compile()
    try:
        for n in (1, 4, 64, 256):
            assert ray.get(cdag.execute(n), timeout=60) == float(n * n * 1024)
    finally:
        cdag.teardown()
