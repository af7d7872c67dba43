"""Tune / Train semantics (modelled on python/ray/tune/tests/test_tuner.py,
test_trial_scheduler.py, test_result_grid.py, test_tune_restore.py and
python/ray/train/tests/test_data_parallel_trainer.py, test_checkpoint_manager.py)."""

import os

import numpy as np
import pytest

import ray_amd as ray
from ray_amd import train, tune
from ray_amd.train import CheckpointConfig, RunConfig, ScalingConfig


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _quad(config):
    for i in range(5):
        train.report({"score": -(config["x"] - 3) ** 2 + i * 0.01, "it": i})


def test_result_grid_best_and_dataframe(cluster, tmp_path):
    tuner = tune.Tuner(_quad, param_space={"x": tune.grid_search([0, 1, 2, 3, 4, 5])},
                       tune_config=tune.TuneConfig(metric="score", mode="max"),
                       run_config=RunConfig(storage_path=str(tmp_path), name="q"))
    grid = tuner.fit()
    assert len(grid) == 6 and grid.num_errors == 0
    best = grid.get_best_result()
    assert best.config["x"] == 3
    worst = grid.get_best_result(metric="score", mode="min")
    assert worst.config["x"] in (0,)
    df = grid.get_dataframe()
    assert len(df) == 6 and "score" in df.columns
    assert all(r.metrics["it"] == 4 for r in grid)


def test_trial_errors_are_collected_not_raised(cluster, tmp_path):
    def fn(config):
        if config["x"] == 1:
            raise ValueError("bad trial")
        train.report({"score": config["x"]})

    grid = tune.Tuner(fn, param_space={"x": tune.grid_search([0, 1, 2])},
                      tune_config=tune.TuneConfig(metric="score", mode="max"),
                      run_config=RunConfig(storage_path=str(tmp_path), name="e")).fit()
    assert grid.num_errors == 1
    assert len(grid.errors) == 1 and "bad trial" in str(grid.errors[0])
    assert grid.get_best_result().config["x"] == 2


def test_num_samples_with_random_space_and_seed_reproducible(cluster, tmp_path):
    def fn(config):
        train.report({"v": config["a"] + config["b"]})

    space = {"a": tune.uniform(0, 1), "b": tune.choice([10, 20, 30])}
    g = tune.Tuner(fn, param_space=space,
                   tune_config=tune.TuneConfig(num_samples=8, metric="v", mode="max"),
                   run_config=RunConfig(storage_path=str(tmp_path), name="r")).fit()
    cfgs = [r.config for r in g]
    assert len(cfgs) == 8
    assert all(0 <= c["a"] <= 1 and c["b"] in (10, 20, 30) for c in cfgs)


def test_stop_criteria_dict(cluster, tmp_path):
    def fn(config):
        for i in range(100):
            train.report({"it": i})

    g = tune.Tuner(fn, param_space={},
                   run_config=RunConfig(storage_path=str(tmp_path), name="s",
                                        stop={"it": 4})).fit()
    assert g[0].metrics["it"] == 4


def test_median_stopping_rule_cuts_losers(cluster, tmp_path):
    from ray_amd.tune.schedulers import MedianStoppingRule

    def fn(config):
        for i in range(30):
            train.report({"acc": config["q"] * (i + 1)})

    sched = MedianStoppingRule(time_attr="training_iteration", grace_period=3,
                               min_samples_required=2)
    # the weak trial comes last, so the others' histories exist when it is judged
    g = tune.Tuner(fn, param_space={"q": tune.grid_search([1.0, 1.1, 1.2, 0.1])},
                   tune_config=tune.TuneConfig(metric="acc", mode="max", scheduler=sched,
                                               # two at a time: the weak trial starts
                                               # after two others finished, however
                                               # loaded the machine is
                                               max_concurrent_trials=2),
                   run_config=RunConfig(storage_path=str(tmp_path), name="m")).fit()
    iters = {r.config["q"]: r.metrics["training_iteration"] for r in g}
    assert iters[0.1] < 30 and iters[1.2] == 30


def test_trainer_keeps_top_k_checkpoints(cluster, tmp_path):
    def loop(config):
        import tempfile

        for i in range(5):
            d = tempfile.mkdtemp()
            with open(os.path.join(d, "step"), "w") as f:
                f.write(str(i))
            train.report({"loss": [5, 1, 4, 2, 3][i], "i": i},
                         checkpoint=train.Checkpoint.from_directory(d))

    from ray_amd.train.data_parallel_trainer import DataParallelTrainer

    res = DataParallelTrainer(
        loop, scaling_config=ScalingConfig(num_workers=1),
        run_config=RunConfig(storage_path=str(tmp_path), name="ck",
                             checkpoint_config=CheckpointConfig(
                                 num_to_keep=2, checkpoint_score_attribute="loss",
                                 checkpoint_score_order="min"))).fit()
    kept = sorted(int(open(os.path.join(c.path, "step")).read())
                  for c, _ in res.best_checkpoints)
    # the two best (losses 1 and 2: steps 1, 3) plus the latest (step 4), as the reference
    assert kept == [1, 3, 4]
    assert int(open(os.path.join(res.checkpoint.path, "step")).read()) == 4


def test_world_rank_and_size_in_context(cluster, tmp_path):
    from ray_amd.train.data_parallel_trainer import DataParallelTrainer

    def loop(config):
        ctx = train.get_context()
        train.report({"rank": ctx.get_world_rank(), "size": ctx.get_world_size(),
                      "local": ctx.get_local_rank()})

    res = DataParallelTrainer(loop, scaling_config=ScalingConfig(num_workers=3),
                              run_config=RunConfig(storage_path=str(tmp_path),
                                                   name="ctx")).fit()
    assert res.metrics["size"] == 3 and res.metrics["rank"] == 0


def test_tuner_over_trainer(cluster, tmp_path):
    """Tune driving a Train trainer (reference: Tuner(trainer, param_space=
    {"train_loop_config": ...}))."""
    from ray_amd.train.data_parallel_trainer import DataParallelTrainer

    def loop(config):
        train.report({"obj": -abs(config["lr"] - 0.1)})

    trainer = DataParallelTrainer(loop, scaling_config=ScalingConfig(num_workers=1),
                                  run_config=RunConfig(storage_path=str(tmp_path), name="t"))
    g = tune.Tuner(trainer,
                   param_space={"train_loop_config": {"lr": tune.grid_search([0.01, 0.1, 1.0])}},
                   tune_config=tune.TuneConfig(metric="obj", mode="max")).fit()
    assert np.isclose(g.get_best_result().config["train_loop_config"]["lr"], 0.1)
