"""Ray Data -> GPU ingest: iter_torch_batches(device="cuda") feeding the HIP
preprocessing kernel (BASELINE config 4 path; reference:
python/ray/data/tests/test_iterator.py torch-batches-on-device cases)."""

import numpy as np
import pytest
import torch

import ray_amd as ray
import ray_amd.data as rd
from ray_amd.ops import functional as rf
from ray_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4, num_gpus=1)
    yield
    ray.shutdown()


def _images(batch):
    ids = batch["id"]
    rng = np.random.default_rng(int(ids[0]))
    return {"image": rng.integers(0, 256, size=(len(ids), 64, 64, 3), dtype=np.uint8),
            "label": ids.astype(np.int64)}


def test_iter_torch_batches_cuda_feeds_hip_normalize(cluster):
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    ds = rd.range(256, override_num_blocks=8).map_batches(_images, batch_size=32)
    expected = {int(b["label"][0]): b["image"] for b in ds.iter_batches(batch_size=32)}
    seen = 0
    for b in ds.iter_torch_batches(batch_size=32, device="cuda", drop_last=True):
        img = b["image"]
        assert img.is_cuda and img.dtype == torch.uint8 and img.shape == (32, 64, 64, 3)
        y = rf.image_normalize(img, mean, std, torch.bfloat16)
        want = ref.image_normalize(torch.from_numpy(expected[int(b["label"][0])]), mean, std)
        assert torch.allclose(y.float().cpu(), want, atol=2e-2, rtol=8e-3)
        seen += img.shape[0]
    assert seen == 256


def test_gpu_preprocessor_actor_pool(cluster):
    from ray_amd.data.preprocessors import GPUImageNormalize

    ds = rd.range(64, override_num_blocks=4).map_batches(_images, batch_size=16)
    out = GPUImageNormalize(out_dtype="fp32", batch_size=16).transform(ds)
    rows = out.take_batch(16)
    x = next(iter(ds.iter_batches(batch_size=16)))["image"]
    want = ref.image_normalize(torch.from_numpy(x), (0.485, 0.456, 0.406),
                               (0.229, 0.224, 0.225))
    assert np.allclose(rows["image"], want.numpy(), atol=1e-4)


def test_device_blocks_through_hbm_store(cluster):
    """GPU actor-pool preprocessing keeps its output on the device: blocks travel through
    the HBM object store and reach iter_torch_batches(device="cuda") with no H2D."""
    from ray_amd.data.preprocessors import GPUImageNormalize

    ds = rd.range(128, override_num_blocks=4).map_batches(_images, batch_size=32)
    out = GPUImageNormalize(out_dtype="bf16", batch_size=32, num_gpus=0.5,
                            keep_on_device=True).transform(ds)
    n = 0
    for b in out.iter_torch_batches(batch_size=32, device="cuda"):
        x = b["image"]
        assert x.is_cuda and x.dtype == torch.bfloat16 and x.shape == (32, 3, 64, 64)
        want = ref.image_normalize(torch.from_numpy(_images({"id": b["label"].cpu().numpy()})
                                                    ["image"]), (0.485, 0.456, 0.406),
                                   (0.229, 0.224, 0.225))
        assert torch.allclose(x.float().cpu(), want, atol=2e-2, rtol=8e-3)
        n += 32
    assert n == 128
