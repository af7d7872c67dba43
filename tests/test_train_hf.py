"""transformers.Trainer inside TorchTrainer workers (modelled on
python/ray/train/tests/test_transformers_trainer.py): 2 gloo ranks train a tiny
random-init GPT-2 with the HF Trainer (which sees the workers' process group and
uses DDP), RayTrainReportCallback reports every HF checkpoint, and prepare_trainer
feeds a ray_amd Data shard."""

import os

import numpy as np
import pytest

import ray_amd as ray
import ray_amd.data  # noqa: F401
from ray_amd.train import RunConfig, ScalingConfig
from ray_amd.train.torch import TorchTrainer

transformers = pytest.importorskip("transformers")


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _loop(config):
    import torch
    import transformers as tf

    from ray_amd import train
    from ray_amd.train.huggingface.transformers import RayTrainReportCallback, prepare_trainer

    torch.manual_seed(0)
    model = tf.GPT2LMHeadModel(tf.GPT2Config(vocab_size=64, n_positions=32, n_embd=32,
                                             n_layer=2, n_head=2))
    shard = train.get_dataset_shard("train")
    args = tf.TrainingArguments(
        output_dir=config["out"], max_steps=6, per_device_train_batch_size=4, save_steps=3,
        save_strategy="steps", logging_steps=1, report_to=[], use_cpu=True,
        learning_rate=1e-3, disable_tqdm=True, dataloader_num_workers=0)
    tr = tf.Trainer(model=model, args=args, train_dataset=shard)
    tr.add_callback(RayTrainReportCallback())
    tr = prepare_trainer(tr)
    tr.train()


def test_transformers_trainer_ddp(cluster, tmp_path):
    rng = np.random.default_rng(0)
    toks = rng.integers(0, 64, size=(64, 16)).astype(np.int64)
    ds = ray.data.from_items([{"input_ids": t, "labels": t} for t in toks])
    trainer = TorchTrainer(_loop, train_loop_config={"out": str(tmp_path / "hf")},
                           scaling_config=ScalingConfig(num_workers=2),
                           datasets={"train": ds},
                           run_config=RunConfig(name="hf", storage_path=str(tmp_path / "r")))
    result = trainer.fit()
    assert result.metrics["step"] == 6 and "loss" in result.metrics
    assert len(result.metrics_history) == 2  # one report per HF save (steps 3 and 6)
    assert os.path.exists(os.path.join(result.checkpoint.path, "checkpoint",
                                       "model.safetensors"))
