"""TensorBoard event files from Tune without tensorboardX (modelled on
python/ray/tune/tests/test_logger.py TBX cases). The Event bytes are checked against the
protobuf library's own parser (Event/Summary messages built from a runtime descriptor with
the field numbers of tensorflow/core/util/event.proto and framework/summary.proto)."""

import glob
import os

import pytest

import ray_amd as ray
from ray_amd import tune
from ray_amd.tune.logger import EventFileWriter, read_event_file


def _event_class():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="ev_test.proto", package="tbx",
                                             syntax="proto3")
    summ = fdp.message_type.add(name="Summary")
    val = summ.nested_type.add(name="Value")
    val.field.add(name="tag", number=1, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
    val.field.add(name="simple_value", number=2, type=F.TYPE_FLOAT, label=F.LABEL_OPTIONAL)
    summ.field.add(name="value", number=1, type=F.TYPE_MESSAGE, label=F.LABEL_REPEATED,
                   type_name=".tbx.Summary.Value")
    ev = fdp.message_type.add(name="Event")
    ev.field.add(name="wall_time", number=1, type=F.TYPE_DOUBLE, label=F.LABEL_OPTIONAL)
    ev.field.add(name="step", number=2, type=F.TYPE_INT64, label=F.LABEL_OPTIONAL)
    ev.field.add(name="file_version", number=3, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
    ev.field.add(name="summary", number=5, type=F.TYPE_MESSAGE, label=F.LABEL_OPTIONAL,
                 type_name=".tbx.Summary")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("tbx.Event"))


def test_event_file_parses_with_protobuf(tmp_path):
    from ray_amd._native import _core

    w = EventFileWriter(str(tmp_path))
    w.add_scalars(3, [("loss", 0.25), ("acc", 0.75)])
    w.close()
    data = open(w.path, "rb").read()
    Event = _event_class()
    evs = [Event.FromString(data[o:o + n]) for o, n in _core.tfrecord_index(data, True)]
    assert evs[0].file_version == "brain.Event:2"
    assert evs[1].step == 3 and evs[1].wall_time > 1e9
    assert {v.tag: v.simple_value for v in evs[1].summary.value} == {"loss": 0.25,
                                                                    "acc": 0.75}


def test_tune_writes_tensorboard_scalars(tmp_path):
    ray.init(num_cpus=2)
    try:
        def trainable(config):
            for i in range(3):
                tune.report({"score": config["x"] * (i + 1), "nested": {"m": float(i)}})

        tuner = tune.Tuner(trainable, param_space={"x": tune.grid_search([1, 2])},
                           run_config=tune.RunConfig(storage_path=str(tmp_path), name="tb"))
        grid = tuner.fit()
        assert not grid.errors
        files = glob.glob(os.path.join(str(tmp_path), "tb", "*", "events.out.tfevents.*"))
        assert len(files) == 2
        seen = {}
        for f in files:
            evs = read_event_file(f)
            assert evs[0][2] == "brain.Event:2"
            x = next(t["config/x"] for _, t, _ in evs if "config/x" in t)
            scores = {step: t["ray/tune/score"] for step, t, _ in evs if "ray/tune/score" in t}
            seen[x] = scores
            assert all("ray/tune/nested/m" in t for _, t, _ in evs if "ray/tune/score" in t)
        assert seen == {1.0: {1: 1.0, 2: 2.0, 3: 3.0}, 2.0: {1: 2.0, 2: 4.0, 3: 6.0}}
    finally:
        ray.shutdown()


def test_pbt_exploits_class_trainables_without_checkpoint_frequency(tmp_path):
    """PBT makes top class-trainable trials checkpoint at their perturbation interval, so
    bottom trials can clone them even when no checkpoint_frequency is configured."""
    from ray_amd.tune.schedulers import PopulationBasedTraining

    class Climb(tune.Trainable):
        def setup(self, config):
            self.value = 0.0
            self.restored_from = None

        def step(self):
            import time

            time.sleep(0.1)  # both trials run side by side (PBT ranks live trials)
            self.value += self.config["lr"]
            return {"score": self.value, "restored": self.restored_from is not None}

        def save_checkpoint(self, d):
            return {"value": self.value}

        def load_checkpoint(self, state):
            self.value = state["value"]
            self.restored_from = state

    ray.init(num_cpus=4)
    try:
        pbt = PopulationBasedTraining(time_attr="training_iteration", metric="score",
                                      mode="max", perturbation_interval=2,
                                      hyperparam_mutations={"lr": [0.1, 1.0, 10.0]},
                                      quantile_fraction=0.5, seed=0)
        grid = tune.Tuner(
            Climb, param_space={"lr": tune.grid_search([0.1, 10.0])},
            tune_config=tune.TuneConfig(scheduler=pbt, metric="score", mode="max"),
            run_config=tune.RunConfig(stop={"training_iteration": 8},
                                      storage_path=str(tmp_path), name="pbtc")).fit()
        assert not grid.errors
        assert pbt.num_perturbations >= 1
        # the slow trial cloned the fast one's state: it ends far above 8 * 0.1
        assert min(r.metrics["score"] for r in grid) > 8 * 0.1 + 1.0
    finally:
        ray.shutdown()
