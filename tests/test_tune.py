"""Tune tests (modelled on python/ray/tune/tests/test_tuner.py, test_trial_scheduler.py,
test_sample.py)."""

import math
import os
import time

import pytest

import ray_amd as ray
from ray_amd import train, tune
from ray_amd.tune.schedulers import AsyncHyperBandScheduler, PopulationBasedTraining


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def objective(config):
    for i in range(10):
        train.report({"score": config["a"] * (i + 1) + config.get("b", 0)})


def test_grid_and_random(cluster, tmp_path):
    tuner = tune.Tuner(objective,
                       param_space={"a": tune.grid_search([1, 2, 3]),
                                    "b": tune.uniform(0, 1)},
                       tune_config=tune.TuneConfig(metric="score", mode="max", num_samples=2),
                       run_config=tune.RunConfig(storage_path=str(tmp_path), name="g"))
    rg = tuner.fit()
    assert len(rg) == 6 and rg.num_errors == 0
    best = rg.get_best_result()
    assert best.config["a"] == 3 and best.metrics["training_iteration"] == 10
    df = rg.get_dataframe()
    assert len(df) == 6 and "config/a" in df.columns


def test_asha_stops_bad_trials(cluster, tmp_path):
    def f(config):
        for i in range(20):
            train.report({"acc": config["q"] * i})

    # best trials first: ASHA can only cut a trial that is below the top 1/rf of the
    # trials already recorded at a rung
    rg = tune.Tuner(f, param_space={"q": tune.grid_search([5.0, 4.0, 3.0, 2.0, 1.0, 0.5, 0.2,
                                                           0.1])},
                    tune_config=tune.TuneConfig(metric="acc", mode="max", scheduler=
                                                AsyncHyperBandScheduler(max_t=20,
                                                                        grace_period=2,
                                                                        reduction_factor=2),
                                                max_concurrent_trials=8),
                    run_config=tune.RunConfig(storage_path=str(tmp_path))).fit()
    iters = sorted(r.metrics["training_iteration"] for r in rg)
    assert iters[0] < 20 and iters[-1] >= 19


class MyTrainable(tune.Trainable):
    def setup(self, config):
        self.x = 0
        self.lr = config["lr"]

    def step(self):
        self.x += self.lr
        return {"x": self.x}

    def save_checkpoint(self, d):
        return {"x": self.x}

    def load_checkpoint(self, state):
        self.x = state["x"]


def test_class_trainable_and_stop(cluster, tmp_path):
    rg = tune.Tuner(MyTrainable, param_space={"lr": tune.choice([1.0, 2.0])},
                    tune_config=tune.TuneConfig(num_samples=2),
                    run_config=tune.RunConfig(stop={"training_iteration": 5},
                                              storage_path=str(tmp_path))).fit()
    assert all(r.metrics["training_iteration"] == 5 for r in rg)


def test_pbt_exploits(cluster, tmp_path):
    def f(config):
        step = 0
        val = 0.0
        ck = train.get_checkpoint()
        if ck:
            with open(os.path.join(ck.path, "s")) as fh:
                step, val = map(float, fh.read().split())
        while step < 12:
            step += 1
            val += config["lr"]
            time.sleep(0.05)  # keep the population concurrent (PBT compares live trials)
            d = os.path.join(config["tmp"], f"{os.getpid()}_{step}_{config['lr']}")
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, "s"), "w") as fh:
                fh.write(f"{step} {val}")
            train.report({"val": val}, checkpoint=tune.Checkpoint(d))

    pbt = PopulationBasedTraining(metric="val", mode="max", perturbation_interval=3,
                                  hyperparam_mutations={"lr": [0.01, 0.1, 1.0, 2.0]}, seed=0)
    rg = tune.Tuner(f, param_space={"lr": tune.grid_search([0.01, 0.1, 1.0, 2.0]),
                                    "tmp": str(tmp_path)},
                    tune_config=tune.TuneConfig(scheduler=pbt, max_concurrent_trials=4),
                    run_config=tune.RunConfig(storage_path=str(tmp_path / "r"))).fit()
    assert pbt.num_perturbations > 0
    assert rg.get_best_result("val", "max").metrics["val"] > 1.0


def test_tune_run_legacy(cluster, tmp_path):
    a = tune.run(objective, config={"a": tune.grid_search([1, 2])}, metric="score", mode="max",
                 storage_path=str(tmp_path))
    assert a.best_config["a"] == 2


def test_sample_domains():
    from ray_amd.tune.search.sample import generate_variants

    vs = list(generate_variants({"x": tune.randint(0, 5), "y": tune.loguniform(1e-4, 1e-1),
                                 "z": tune.grid_search(["a", "b"]),
                                 "w": tune.sample_from(lambda spec: spec.config["x"] * 2)},
                                num_samples=3, seed=0))
    assert len(vs) == 6
    assert all(0 <= v["x"] < 5 and 1e-4 <= v["y"] <= 1e-1 and v["w"] == 2 * v["x"] for v in vs)


def _ckpt_trainable(config):
    step, val = 0, 0.0
    ck = train.get_checkpoint()
    if ck:
        with open(os.path.join(ck.path, "s")) as fh:
            step, val = map(float, fh.read().split())
    while step < 12:
        step += 1
        val += config["lr"]
        time.sleep(0.05)
        d = os.path.join(config["tmp"], f"{os.getpid()}_{step}_{config['lr']}_{time.time()}")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "s"), "w") as fh:
            fh.write(f"{step} {val}")
        cpus = ray.get_runtime_context().get_assigned_resources().get("CPU", 0)
        train.report({"val": val, "cpus": cpus}, checkpoint=tune.Checkpoint(d))


def test_pb2_gp_explore(cluster, tmp_path):
    from ray_amd.tune.schedulers import PB2

    pb2 = PB2(metric="val", mode="max", perturbation_interval=3,
              hyperparam_bounds={"lr": [0.01, 2.0]}, seed=0)
    rg = tune.Tuner(_ckpt_trainable,
                    param_space={"lr": tune.grid_search([0.01, 0.05, 1.0, 2.0]),
                                 "tmp": str(tmp_path)},
                    tune_config=tune.TuneConfig(scheduler=pb2, max_concurrent_trials=4),
                    run_config=tune.RunConfig(storage_path=str(tmp_path / "r"))).fit()
    assert pb2.num_perturbations > 0 and len(pb2.data) > 0
    assert rg.get_best_result("val", "max").metrics["val"] > 1.0
    # explored configs stay inside the bounds
    for r in rg:
        assert 0.01 <= r.config["lr"] <= 2.0


def test_resource_changing_scheduler(cluster, tmp_path):
    from ray_amd.tune.schedulers import ResourceChangingScheduler

    sched = ResourceChangingScheduler()
    rg = tune.Tuner(_ckpt_trainable,
                    param_space={"lr": tune.grid_search([0.1, 0.2]), "tmp": str(tmp_path)},
                    tune_config=tune.TuneConfig(scheduler=sched, metric="val", mode="max",
                                                max_concurrent_trials=2),
                    run_config=tune.RunConfig(storage_path=str(tmp_path / "r"))).fit()
    # 4 CPUs over 2 trials: both grow from 1 to 2 CPUs (checkpoint + restart) and finish
    assert sched.num_reallocations >= 2
    assert all(abs(r.metrics["val"] - 12 * r.config["lr"]) < 1e-6 for r in rg)
    assert all(r.metrics["cpus"] >= 2 for r in rg), [r.metrics for r in rg]


# ---------------------------------------------------------------- model-based searchers
# (reference: python/ray/tune/tests/test_searchers.py drives each adapter through Tuner)

def _drive(searcher, space, f, n, mode="min"):
    searcher.set_search_properties("loss", mode, space)
    best = None
    for i in range(n):
        cfg = searcher.suggest(str(i))
        v = f(cfg)
        searcher.on_trial_complete(str(i), {"loss": v})
        best = v if best is None else (min(best, v) if mode == "min" else max(best, v))
    return best


def test_tpe_beats_random_on_quadratic():
    from ray_amd.tune.search import TPESearch
    space = {"x": tune.uniform(-5, 5), "y": tune.loguniform(1e-3, 1.0),
             "opt": tune.choice(["sgd", "adam"]), "const": 7}

    def f(c):
        assert c["const"] == 7
        return (c["x"] - 1.5) ** 2 + abs(math.log10(c["y"]) + 2) + (c["opt"] != "adam")

    tpe = [_drive(TPESearch(seed=s, n_initial_points=8), space, f, 60) for s in range(4)]
    import random
    rnd = []
    for s in range(4):
        rng = random.Random(s)
        rnd.append(min(f({"x": rng.uniform(-5, 5), "y": 10 ** rng.uniform(-3, 0),
                          "opt": rng.choice(["sgd", "adam"]), "const": 7}) for _ in range(60)))
    assert sum(tpe) / 4 < sum(rnd) / 4
    assert max(tpe) < 0.5


def test_bayesopt_finds_max_and_rejects_categorical():
    from ray_amd.tune.search import BayesOptSearch
    space = {"a": tune.uniform(0, 1), "b": tune.uniform(-2, 2)}
    best = _drive(BayesOptSearch(random_state=0, random_search_steps=5), space,
                  lambda c: -((c["a"] - 0.3) ** 2) - (c["b"] - 1.0) ** 2, 25, mode="max")
    assert best > -0.02
    ei = _drive(BayesOptSearch(random_state=1, random_search_steps=5,
                               utility_kwargs={"kind": "ei", "xi": 0.0}), space,
                lambda c: (c["a"] - 0.3) ** 2 + (c["b"] - 1.0) ** 2, 25)
    assert ei < 0.05
    with pytest.raises(ValueError):
        BayesOptSearch(space={"c": tune.choice([1, 2])})


def test_tuner_with_tpe_respects_num_samples(cluster, tmp_path):
    from ray_amd.tune.search import ConcurrencyLimiter, HyperOptSearch

    def obj(config):
        train.report({"loss": (config["x"] - 2.0) ** 2})

    alg = ConcurrencyLimiter(HyperOptSearch(n_initial_points=4, seed=0), max_concurrent=2)
    rg = tune.Tuner(obj, param_space={"x": tune.uniform(-4, 4)},
                    tune_config=tune.TuneConfig(metric="loss", mode="min", num_samples=12,
                                                search_alg=alg),
                    run_config=tune.RunConfig(storage_path=str(tmp_path), name="tpe")).fit()
    assert len(rg) == 12 and rg.num_errors == 0
    assert rg.get_best_result().metrics["loss"] < 1.0
