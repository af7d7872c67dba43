"""Tune progress reporting (reference: python/ray/tune/tests/test_progress_reporter.py):
RunConfig.progress_reporter receives the trials during and at the end of the run, the
default CLIReporter prints the final status table, verbose=0 prints nothing."""
import pytest

import ray_amd as ray
from ray_amd import tune
from ray_amd.train import RunConfig
from ray_amd.tune.registry import ProgressReporter


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _trainable(config):
    for i in range(3):
        tune.report({"score": config["x"] * i})


def test_custom_reporter_called(cluster, tmp_path):
    calls = []

    class Rec(ProgressReporter):
        def report(self, trials, done, *sys_info):
            calls.append((done, sorted(t.status for t in trials)))

    tune.Tuner(_trainable, param_space={"x": tune.grid_search([1, 2])},
               run_config=RunConfig(name="rep", storage_path=str(tmp_path),
                                    progress_reporter=Rec())).fit()
    assert calls and calls[-1] == (True, ["TERMINATED", "TERMINATED"])
    assert any(not d for d, _ in calls)


def test_default_table_and_verbose_zero(cluster, tmp_path, capsys):
    tune.Tuner(_trainable, param_space={"x": tune.grid_search([3])},
               tune_config=tune.TuneConfig(metric="score", mode="max"),
               run_config=RunConfig(name="v1", storage_path=str(tmp_path))).fit()
    out = capsys.readouterr().out
    assert "== Status (done" in out and "score" in out
    tune.Tuner(_trainable, param_space={"x": tune.grid_search([3])},
               run_config=RunConfig(name="v0", storage_path=str(tmp_path), verbose=0)).fit()
    assert "== Status" not in capsys.readouterr().out
