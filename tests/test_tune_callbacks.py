"""Tune callbacks / loggers and Trainer callbacks + restore (modelled on
python/ray/tune/tests/test_callbacks.py, test_logger.py and
python/ray/train/tests/test_trainer_restore.py)."""

import csv
import json
import os

import pytest

import ray_amd as ray
from ray_amd import train, tune
from ray_amd.train import Checkpoint, CheckpointConfig, FailureConfig, RunConfig, ScalingConfig
from ray_amd.train.torch import TorchTrainer


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


class Recorder(tune.Callback):
    def __init__(self):
        self.events = []

    def setup(self, **info):
        self.events.append(("setup", None))

    def on_trial_start(self, iteration, trials, trial, **info):
        self.events.append(("start", trial.trial_id))

    def on_trial_result(self, iteration, trials, trial, result, **info):
        self.events.append(("result", result.get("score")))

    def on_checkpoint(self, iteration, trials, trial, checkpoint, **info):
        self.events.append(("ckpt", os.path.basename(checkpoint.path)))

    def on_trial_complete(self, iteration, trials, trial, **info):
        self.events.append(("complete", trial.trial_id))

    def on_trial_error(self, iteration, trials, trial, **info):
        self.events.append(("error", trial.trial_id))

    def on_experiment_end(self, trials, **info):
        self.events.append(("end", len(trials)))


class Broken(tune.Callback):
    def on_trial_result(self, *a, **k):
        raise RuntimeError("callback bug")


def objective(config):
    for i in range(3):
        train.report({"score": config["a"] * (i + 1), "nested": {"x": i}})


def test_tuner_callbacks_and_default_loggers(cluster, tmp_path):
    rec = Recorder()
    rg = tune.Tuner(objective, param_space={"a": tune.grid_search([1, 2])},
                    run_config=tune.RunConfig(storage_path=str(tmp_path), name="cb",
                                              callbacks=[rec, Broken()])).fit()
    assert rg.num_errors == 0  # a raising callback is disabled, not fatal
    kinds = [k for k, _ in rec.events]
    assert kinds[0] == "setup" and kinds[-1] == "end"
    assert kinds.count("start") == 2 and kinds.count("complete") == 2
    assert sorted(v for k, v in rec.events if k == "result") == [1, 2, 2, 3, 4, 6]
    for r in rg:
        d = r.path
        rows = list(csv.DictReader(open(os.path.join(d, "progress.csv"))))
        assert len(rows) == 3 and "nested/x" in rows[0] and rows[-1]["nested/x"] == "2"
        lines = [json.loads(x) for x in open(os.path.join(d, "result.json"))]
        assert [x["score"] for x in lines] == [r.config["a"] * i for i in (1, 2, 3)]
        assert json.load(open(os.path.join(d, "params.json"))) == r.config


def test_trainer_fires_run_config_callbacks(cluster, tmp_path):
    rec = Recorder()

    def loop(config):
        import tempfile

        for i in range(3):
            d = tempfile.mkdtemp()
            with open(os.path.join(d, "w.json"), "w") as f:
                json.dump({"i": i}, f)
            train.report({"score": i}, checkpoint=Checkpoint(d))

    TorchTrainer(loop, scaling_config=ScalingConfig(num_workers=2),
                 run_config=RunConfig(storage_path=str(tmp_path), name="tr",
                                      callbacks=[rec])).fit()
    assert [v for k, v in rec.events if k == "result"] == [0, 1, 2]
    assert [v for k, v in rec.events if k == "ckpt"] == [
        "checkpoint_000000", "checkpoint_000001", "checkpoint_000002"]
    assert ("complete", "tr") in rec.events
    rows = list(csv.DictReader(open(os.path.join(tmp_path, "tr", "progress.csv"))))
    assert [r["score"] for r in rows] == ["0", "1", "2"]


def _resumable_loop(config):
    import tempfile

    start = 0
    ck = train.get_checkpoint()
    if ck is not None:
        with open(os.path.join(ck.path, "state.json")) as f:
            start = json.load(f)["i"] + 1
    for i in range(start, 5):
        if i == 3 and config["crash"] and ck is None:
            raise RuntimeError("simulated node failure")
        d = tempfile.mkdtemp()
        with open(os.path.join(d, "state.json"), "w") as f:
            json.dump({"i": i}, f)
        train.report({"i": i, "resumed_from": start}, checkpoint=Checkpoint(d))


def test_trainer_restore_resumes_from_latest_checkpoint(cluster, tmp_path):
    trainer = TorchTrainer(_resumable_loop, train_loop_config={"crash": True},
                           scaling_config=ScalingConfig(num_workers=1),
                           run_config=RunConfig(storage_path=str(tmp_path), name="rs",
                                                failure_config=FailureConfig(max_failures=0),
                                                checkpoint_config=CheckpointConfig(
                                                    num_to_keep=2)))
    with pytest.raises(train.TrainingFailedError):
        trainer.fit()
    path = os.path.join(tmp_path, "rs")
    assert TorchTrainer.can_restore(path)
    restored = TorchTrainer.restore(path)
    assert restored.resume_from_checkpoint is not None
    res = restored.fit()
    assert res.metrics["i"] == 4 and res.metrics["resumed_from"] == 3
    # a run that needs datasets must get them again
    assert not TorchTrainer.can_restore(str(tmp_path / "nope"))
