"""Data all-to-all operators in the streaming executor: zip aligned to the left block
boundaries (reference operators/zip_operator.py:19), streaming union (union_operator.py:12),
dynamic block splitting by target_max_block_size (map_operator.py:53) and push-based shuffle
(push_based_shuffle_task_scheduler.py:400)."""
import time

import numpy as np
import pytest

import ray_amd as ray
from ray_amd import data
from ray_amd.data import DataContext


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=8)
    yield
    ray.shutdown()


def test_zip_keeps_left_block_boundaries(cluster):
    a = data.range(640, override_num_blocks=64)
    b = data.range(640, override_num_blocks=7).map_batches(lambda x: {"y": x["id"] * 10})
    z = a.zip(b).materialize()
    assert z.num_blocks() == 64
    rows = z.take_all()
    assert len(rows) == 640 and all(r["y"] == 10 * r["id"] for r in rows)
    z2 = data.range(100, override_num_blocks=3).zip(data.range(100, override_num_blocks=64))
    assert z2.materialize().num_blocks() == 3
    assert [r["id_1"] for r in z2.take_all()] == list(range(100))


def test_zip_row_count_mismatch(cluster):
    with pytest.raises(Exception, match="different number of rows"):
        data.range(10).zip(data.range(11)).materialize()
    with pytest.raises(Exception, match="different number of rows"):
        data.range(11).zip(data.range(10)).materialize()


def test_union_streams_without_materialising(cluster):
    def slow(b):
        time.sleep(1.0)
        return b

    fast = data.range(8, override_num_blocks=4)
    slow_ds = data.range(8, override_num_blocks=4).map_batches(slow, concurrency=1)
    u = fast.union(slow_ds, data.range(3, override_num_blocks=1))
    t0 = time.time()
    it = iter(u.iter_batches(batch_size=None))
    first = next(it)
    t_first = time.time() - t0
    rest = list(it)
    t_all = time.time() - t0
    assert t_first < 1.0 < t_all  # the fast input streamed out before the slow one ran
    ids = np.concatenate([first["id"]] + [b["id"] for b in rest]).tolist()
    assert ids == list(range(8)) + list(range(8)) + list(range(3))
    assert data.range(5).union(data.range(5)).count() == 10


def test_target_max_block_size_splits_outputs(cluster):
    ctx = DataContext.get_current()
    old = ctx.target_max_block_size
    ctx.target_max_block_size = 32 << 20
    try:
        def big(b):  # one 256 MiB batch from a 1-row input block
            return {"x": np.ones((256 << 20) // 8, dtype=np.float64)}

        ds = data.range(1, override_num_blocks=1).map_batches(big, batch_size=None)
        mat = ds.materialize()
        sizes = [ray.get(r)["x"].nbytes for r in mat.get_internal_block_refs()]
        assert len(sizes) == 8 and max(sizes) <= 32 << 20
        assert sum(sizes) == 256 << 20 and mat.count() == (256 << 20) // 8
    finally:
        ctx.target_max_block_size = old


@pytest.mark.parametrize("push", [False, True])
def test_shuffle_and_sort_push_based(cluster, push):
    ctx = DataContext.get_current()
    old = ctx.use_push_based_shuffle, ctx.push_based_shuffle_merge_factor
    ctx.use_push_based_shuffle, ctx.push_based_shuffle_merge_factor = push, 4
    try:
        ds = data.range(2000, override_num_blocks=20)
        sh = ds.random_shuffle(seed=3, num_blocks=6)
        got = [r["id"] for r in sh.take_all()]
        assert sorted(got) == list(range(2000)) and got != list(range(2000))
        assert sh.materialize().num_blocks() == 6
        srt = ds.random_shuffle(seed=5).sort("id", descending=True)
        assert [r["id"] for r in srt.take_all()] == list(range(1999, -1, -1))
    finally:
        ctx.use_push_based_shuffle, ctx.push_based_shuffle_merge_factor = old


def test_random_shuffle_is_lazy(cluster, tmp_path):
    """random_shuffle() without num_blocks runs nothing upstream until consumption (the
    block count is decided at execution), for a plan that knows its block count (read
    tasks) and for one that does not (a streamed union)."""
    marker = tmp_path / "ran"

    def touch(batch):
        marker.write_text("x")
        return batch

    ds = ray.data.range(1000, override_num_blocks=8).map_batches(touch)
    sh = ds.random_shuffle(seed=3)
    import time

    time.sleep(0.5)
    assert not marker.exists()  # declared, not executed
    rows = [r["id"] for r in sh.iter_rows()]
    assert marker.exists() and sorted(rows) == list(range(1000))
    assert rows != list(range(1000))
    assert sh.materialize().num_blocks() == 8
    u = ray.data.range(10, override_num_blocks=2).union(ray.data.range(10, override_num_blocks=3))
    su = u.random_shuffle(seed=1)
    assert sorted(r["id"] for r in su.iter_rows()) == sorted(list(range(10)) * 2)
