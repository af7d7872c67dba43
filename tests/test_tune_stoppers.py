"""Tune stoppers (reference: python/ray/tune/tests/test_stopper.py): trial plateau with a
metric threshold, experiment plateau over the top-k results, noop, and an experiment the
plateau stopper ends early."""
import pytest

import ray_amd as ray
from ray_amd import tune
from ray_amd.tune.stopper import ExperimentPlateauStopper, NoopStopper, TrialPlateauStopper


def test_trial_plateau_threshold_and_mode():
    s = TrialPlateauStopper("loss", std=0.01, num_results=3, grace_period=3,
                            metric_threshold=0.5, mode="min")
    for v in (1.0, 1.0, 1.0):  # flat but above the threshold (mode min): keep going
        assert not s("t", {"loss": v})
    for v in (0.4, 0.4):
        assert not s("t", {"loss": v})
    assert s("t", {"loss": 0.4})  # last three flat and below the threshold
    assert not s("u", {"other": 1.0})  # results without the metric never stop a trial
    with pytest.raises(ValueError):
        TrialPlateauStopper("loss", metric_threshold=0.1)


def test_experiment_plateau_top_k_and_patience():
    s = ExperimentPlateauStopper("acc", std=0.001, top=3, mode="max", patience=1)
    for v in (0.1, 0.5, 0.9):
        s("a", {"acc": v})
    assert not s.stop_all()
    s("b", {"acc": 0.9}), s("c", {"acc": 0.9})  # top-3 = 0.9, 0.9, 0.9: plateau starts
    assert not s.stop_all()  # within patience
    s("d", {"acc": 0.2})
    assert s.stop_all()
    assert not NoopStopper()("x", {"acc": 1}) and not NoopStopper().stop_all()


def test_experiment_plateau_ends_tuner_early(tmp_path):
    ray.init(num_cpus=4)
    try:
        def trainable(config):
            for i in range(100):
                tune.report({"score": 1.0, "it": i})  # a flat metric from the start

        res = tune.Tuner(
            trainable, param_space={"x": tune.grid_search([1, 2])},
            run_config=tune.RunConfig(
                storage_path=str(tmp_path),
                stop=ExperimentPlateauStopper("score", top=4, mode="max", patience=2)),
        ).fit()
        # the experiment stops once the plateau outlasts the patience: the running trial
        # ends early and a trial still pending never starts
        iters = [r.metrics.get("it", -1) for r in res]
        assert 0 <= max(iters) < 50, iters
    finally:
        ray.shutdown()


def test_trial_name_and_dirname_creators(tmp_path):
    import os

    from ray_amd import train

    ray.init(num_cpus=4)
    try:
        def trainable(config):
            ctx = train.get_context()
            tune.report({"name": ctx.get_trial_name(), "dir": os.path.basename(ctx.get_trial_dir())})

        res = tune.Tuner(
            trainable, param_space={"x": tune.grid_search([1, 2])},
            tune_config=tune.TuneConfig(
                trial_name_creator=lambda t: f"run_x{t.config['x']}",
                trial_dirname_creator=lambda t: f"dir_{t.config['x']}"),
            run_config=tune.RunConfig(storage_path=str(tmp_path)),
        ).fit()
        got = sorted((r.metrics["name"], r.metrics["dir"], os.path.basename(r.path)) for r in res)
        assert got == [("run_x1", "dir_1", "dir_1"), ("run_x2", "dir_2", "dir_2")]
    finally:
        ray.shutdown()


@pytest.mark.parametrize("spec", [True, "out.log"])
def test_log_to_file(tmp_path, spec):
    import os

    ray.init(num_cpus=2)
    try:
        def trainable(config):
            import sys

            print("hello from", config["x"])
            print("warn", config["x"], file=sys.stderr)
            tune.report({"ok": 1})

        res = tune.Tuner(trainable, param_space={"x": 7},
                         run_config=tune.RunConfig(storage_path=str(tmp_path),
                                                   log_to_file=spec)).fit()
        d = res[0].path
        if spec is True:
            assert "hello from 7" in open(os.path.join(d, "stdout")).read()
            assert "warn 7" in open(os.path.join(d, "stderr")).read()
        else:
            txt = open(os.path.join(d, "out.log")).read()
            assert "hello from 7" in txt and "warn 7" in txt
    finally:
        ray.shutdown()


def test_tune_run_raise_on_failed_trial(tmp_path):
    ray.init(num_cpus=2)
    try:
        def bad(config):
            if config["x"] == 2:
                raise ValueError("boom")
            tune.report({"ok": 1})

        with pytest.raises(tune.TuneError, match="1 of 2 errored"):
            tune.run(bad, config={"x": tune.grid_search([1, 2])}, storage_path=str(tmp_path))
        ana = tune.run(bad, config={"x": tune.grid_search([1, 2])}, storage_path=str(tmp_path),
                       raise_on_failed_trial=False, verbose=0)
        assert len(ana.trials) == 2
    finally:
        ray.shutdown()
