"""Public API surface added for parity with the reference's __all__ lists: tune registry /
Experiment / reporters / factories / ResumeConfig / PBT replay, train DataConfig /
TrainingIterator, ray.client, RuntimeEnv, serve.HTTPOptions, the text / hashing / binning
preprocessors and the file datasinks (reference tests: tune/tests/test_api.py,
test_experiment.py, test_progress_reporter.py, train/tests/test_data_parallel_trainer.py,
tests/test_client_builder.py, tests/test_runtime_env.py, data/tests/preprocessors/*)."""

import io
import json
import os

import numpy as np
import pytest

import ray_amd as ray
import ray_amd.data as rd
from ray_amd import train, tune


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _objective(config):
    for i in range(3):
        train.report({"score": config["x"] * (i + 1)})


def test_tune_registry_experiment_reporter(cluster, tmp_path):
    tune.register_trainable("objective", _objective)
    trials = tune.run_experiments(tune.Experiment(
        "exp1", "objective", config={"x": tune.grid_search([1, 2])},
        storage_path=str(tmp_path)))
    assert sorted(t.metrics["score"] for t in trials) == [3, 6]
    ana = tune.run("objective", config={"x": 5}, storage_path=str(tmp_path),
                   resources_per_trial=tune.PlacementGroupFactory([{"CPU": 1}]))
    assert ana.trials[0].metrics["score"] == 15
    with pytest.raises(ValueError):
        tune.Tuner("no_such_trainable")
    rep = tune.CLIReporter(metric_columns=["score"], max_report_frequency=0)

    class _T:
        trial_id, status, config, last_result = "t0", "RUNNING", {"x": 1}, {"score": 3}

    buf = io.StringIO()
    rep._file = buf
    assert rep.should_report([_T()])
    rep.report([_T()], done=False)
    assert "score" in buf.getvalue() and "t0" in buf.getvalue()
    assert type(tune.create_scheduler("asha", metric="score", mode="max")).__name__ == \
        "AsyncHyperBandScheduler"
    assert type(tune.create_searcher("random")).__name__ == "BasicVariantGenerator"
    assert tune.PlacementGroupFactory([{"CPU": 1}, {"GPU": 1}]).required_resources() == \
        {"CPU": 1, "GPU": 1}
    with pytest.raises(ValueError):
        tune.ResumeConfig(unfinished="bogus")


def test_pbt_replay_from_policy_file(tmp_path):
    from ray_amd.tune.schedulers import PopulationBasedTrainingReplay

    f = tmp_path / "pbt_policy_t1.txt"
    f.write_text("\n".join(json.dumps(e) for e in [["t1", "t0", 0, {"lr": 0.1}],
                                                   ["t1", "t2", 4, {"lr": 0.05}]]))
    sched = PopulationBasedTrainingReplay(str(f))

    class Trial:
        config = {}
        last_checkpoint = "ckpt"
        pending_exploit = None

    tr = Trial()
    sched.on_trial_add(None, tr)
    assert tr.config == {"lr": 0.1}
    sched.on_trial_result(None, tr, {"training_iteration": 3})
    assert tr.pending_exploit is None
    sched.on_trial_result(None, tr, {"training_iteration": 4})
    assert tr.pending_exploit == ("ckpt", {"lr": 0.05})


def _loop(config):
    shard = train.get_dataset_shard("valid")
    n = sum(len(b["id"]) for b in shard.iter_batches(batch_size=10))
    for i in range(3):
        train.report({"i": i, "valid_rows": n})


def test_data_config_and_training_iterator(cluster, tmp_path):
    from ray_amd.train import DataConfig, TrainingIterator
    from ray_amd.train.data_parallel_trainer import DataParallelTrainer

    def make(cfg):
        return DataParallelTrainer(
            _loop, scaling_config=train.ScalingConfig(num_workers=2),
            datasets={"valid": rd.range(40)}, dataset_config=cfg,
            run_config=train.RunConfig(storage_path=str(tmp_path)))

    r = make(None).fit()  # default DataConfig: every dataset is split
    assert r.metrics["valid_rows"] == 20
    r = make(DataConfig(datasets_to_split=[])).fit()
    assert r.metrics["valid_rows"] == 40
    it = TrainingIterator(make(None))
    seen = [m["i"] for m in it]
    assert seen[-1] == 2 and it.result.metrics["i"] == 2
    assert train.TRAIN_DATASET_KEY == "train"


def test_text_hash_bin_preprocessors(cluster):
    from ray_amd.data import preprocessors as P

    ds = rd.from_items([{"t": "a b a", "n": 1.0, "c": "x", "tags": ["u", "v"]},
                        {"t": "b c", "n": 5.0, "c": "y", "tags": ["v"]},
                        {"t": "c", "n": 9.0, "c": "x", "tags": []}])
    cv = P.CountVectorizer(["t"]).fit(ds)
    rows = sorted(cv.transform(ds).take_all(), key=lambda r: r["n"])
    assert rows[0]["t_a"] == 2 and rows[0]["t_b"] == 1 and rows[2]["t_c"] == 1
    hv = P.HashingVectorizer(["t"], num_features=8).transform(ds).take_all()
    assert sum(v for k, v in hv[0].items() if k.startswith("hash_t_")) == 3
    fh = P.FeatureHasher(["n", "c"], num_features=4).transform(ds).take_all()
    assert len([k for k in fh[0] if k.startswith("hash_")]) == 4
    tk = P.Tokenizer(["t"]).transform(ds).take_all()
    assert list(tk[0]["t"]) == ["a", "b", "a"]
    mh = P.MultiHotEncoder(["tags"]).fit(ds).transform(ds).take_all()
    assert list(mh[0]["tags"]) == [1, 1] and list(mh[2]["tags"]) == [0, 0]
    rs = P.RobustScaler(["n"]).fit(ds).transform(ds).take_all()
    assert sorted(r["n"] for r in rs) == [-1.0, 0.0, 1.0]
    pt = P.PowerTransformer(["n"], power=0.0).transform(ds).take_all()
    assert abs(sorted(r["n"] for r in pt)[0] - np.log(2.0)) < 1e-9
    ub = P.UniformKBinsDiscretizer(["n"], bins=2).fit(ds).transform(ds).take_all()
    assert sorted(r["n"] for r in ub) == [0.0, 0.0, 1.0]
    cb = P.CustomKBinsDiscretizer(["n"], bins=[0, 2, 6, 10]).transform(ds).take_all()
    assert sorted(r["n"] for r in cb) == [0.0, 1.0, 2.0]
    cz = P.Categorizer(["c"]).fit(ds)
    cat = cz.transform_batch({"c": np.array(["y", "x", "z"], dtype=object)})
    assert str(cat["c"].dtype) == "category" and list(cat["c"].cat.categories) == ["x", "y"]
    assert cat["c"].isna().tolist() == [False, False, True]
    assert sorted(r["c"] for r in cz.transform(ds).take_all()) == ["x", "x", "y"]


class _RowSink(rd.RowBasedFileDatasink):
    def write_row_to_file(self, row, file):
        file.write(json.dumps({"id": int(row["id"])}).encode())


class _BlockSink(rd.BlockBasedFileDatasink):
    def write_block_to_file(self, block, file):
        file.write(str(block.num_rows).encode())


def test_file_datasinks(cluster, tmp_path):
    ds = rd.range(10).repartition(2)
    assert ds.write_datasink(_RowSink(str(tmp_path / "rows"), file_format="json")) == 10
    assert len(os.listdir(tmp_path / "rows")) == 10
    assert ds.write_datasink(_BlockSink(str(tmp_path / "blocks"), file_format="txt")) == 10
    got = sorted(int(open(tmp_path / "blocks" / f).read()) for f in
                 os.listdir(tmp_path / "blocks"))
    assert got == [5, 5]


def test_dag_plot_and_input_data(tmp_path):
    from ray_amd.dag import DAGInputData, InputNode, plot

    @ray.remote
    def inc(x):
        return x + 1

    @ray.remote
    def add(a, b):
        return a + b

    with InputNode() as inp:
        dag = add.bind(inc.bind(inp), inc.bind(inp))
    text = plot(dag, str(tmp_path / "g.dot"))
    assert text.startswith("digraph") and text.count("->") == 4
    assert open(tmp_path / "g.dot").read() == text
    d = DAGInputData(1, 2, k=3)
    assert d[0] == 1 and d["k"] == 3 and d.k == 3
