"""RunConfig.storage_filesystem / URI storage paths (reference: python/ray/train/tests/
test_new_persistence.py): checkpoints are uploaded by the workers into
<storage_path>/<name>/checkpoint_<i> on the given pyarrow filesystem, pruned there, the
driver's result files follow at the end, and checkpoints read back through the fs."""
import json
import os

import pyarrow.fs as pafs
import pytest

import ray_amd as ray
from ray_amd import train
from ray_amd.train import Checkpoint, CheckpointConfig, RunConfig, ScalingConfig
from ray_amd.train.data_parallel_trainer import DataParallelTrainer


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _loop(cfg):
    import tempfile

    for i in range(3):
        d = tempfile.mkdtemp()
        with open(os.path.join(d, f"rank{train.get_context().get_world_rank()}.json"),
                  "w") as f:
            json.dump({"step": i}, f)
        train.report({"step": i, "score": -abs(i - 1)},
                     checkpoint=Checkpoint.from_directory(d))


def test_checkpoints_on_custom_filesystem(cluster, tmp_path, monkeypatch):
    remote = tmp_path / "bucket"
    remote.mkdir()
    monkeypatch.setenv("RAY_AMD_STORAGE", str(tmp_path / "staging"))
    fs = pafs.SubTreeFileSystem(str(remote), pafs.LocalFileSystem())
    t = DataParallelTrainer(
        _loop, scaling_config=ScalingConfig(num_workers=2),
        run_config=RunConfig(name="fsrun", storage_path="exp", storage_filesystem=fs,
                             checkpoint_config=CheckpointConfig(
                                 num_to_keep=1, checkpoint_score_attribute="score")))
    r = t.fit()
    assert r.path == "exp/fsrun" and r.filesystem is fs
    run = remote / "exp" / "fsrun"
    ckpts = sorted(p.name for p in run.iterdir() if p.name.startswith("checkpoint_"))
    # num_to_keep=1 by score keeps the best (step 1) and the latest (step 2)
    assert ckpts == ["checkpoint_000001", "checkpoint_000002"]
    assert sorted(os.listdir(run / "checkpoint_000002")) == ["rank0.json", "rank1.json"]
    assert (run / "result.json").exists()  # driver files uploaded at the end
    c = r.checkpoint
    assert c.filesystem is fs and c.path == "exp/fsrun/checkpoint_000002"
    with c.as_directory() as d:
        assert not d.startswith(str(remote))  # a local download
        assert json.load(open(os.path.join(d, "rank1.json"))) == {"step": 2}
    c.set_metadata({"k": 1})
    assert c.get_metadata() == {"k": 1}
    assert (run / "checkpoint_000002" / ".metadata.json").exists()


def test_file_uri_storage_is_local(cluster, tmp_path):
    t = DataParallelTrainer(
        _loop, scaling_config=ScalingConfig(num_workers=1),
        run_config=RunConfig(name="urirun", storage_path=f"file://{tmp_path}/u"))
    r = t.fit()
    assert r.filesystem is None and r.path == f"{tmp_path}/u/urirun"
    assert r.checkpoint.filesystem is None
    assert os.path.exists(os.path.join(r.checkpoint.path, "rank0.json"))


def test_tune_experiment_uploaded_to_filesystem(cluster, tmp_path, monkeypatch):
    from ray_amd import tune

    remote = tmp_path / "bucket"
    remote.mkdir()
    monkeypatch.setenv("RAY_AMD_STORAGE", str(tmp_path / "staging"))
    fs = pafs.SubTreeFileSystem(str(remote), pafs.LocalFileSystem())

    def trainable(config):
        import tempfile

        for i in range(2):
            d = tempfile.mkdtemp()
            with open(os.path.join(d, "w.txt"), "w") as f:
                f.write(str(config["x"] * 10 + i))
            tune.report({"v": config["x"] + i}, checkpoint=Checkpoint.from_directory(d))

    grid = tune.Tuner(trainable, param_space={"x": tune.grid_search([1, 2])},
                      tune_config=tune.TuneConfig(metric="v", mode="max"),
                      run_config=RunConfig(name="tfs", storage_path="tx",
                                           storage_filesystem=fs)).fit()
    assert grid.experiment_path == "tx/tfs"
    assert (remote / "tx" / "tfs" / "experiment_state.pkl").exists()
    best = grid.get_best_result()
    assert best.filesystem is fs and best.path.startswith("tx/tfs/")
    with best.checkpoint.as_directory() as d:
        assert open(os.path.join(d, "w.txt")).read() == "21"
