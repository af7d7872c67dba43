"""Ray Train tests on CPU (gloo, 2 workers) — modelled on python/ray/train/tests/
test_torch_trainer.py, test_data_parallel_trainer.py, test_checkpoint_manager.py."""

import os

import pytest
import torch

import ray_amd as ray
from ray_amd import train
from ray_amd.train import Checkpoint, CheckpointConfig, FailureConfig, RunConfig, ScalingConfig
from ray_amd.train.torch import TorchTrainer


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _loop(config):
    import torch.distributed as dist

    from ray_amd.train import torch as rt

    ctx = train.get_context()
    torch.manual_seed(0)
    model = torch.nn.Linear(4, 1)
    model = rt.prepare_model(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    x = torch.randn(64, 4)
    y = x.sum(1, keepdim=True)
    start = 0
    ck = train.get_checkpoint()
    if ck is not None:
        start = torch.load(os.path.join(ck.path, "state.pt"))["epoch"] + 1
    for epoch in range(start, config["epochs"]):
        loss = torch.nn.functional.mse_loss(model(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        w = model.module.weight.detach().clone() if hasattr(model, "module") else \
            model.weight.detach().clone()
        if dist.is_initialized():
            ws = [torch.zeros_like(w) for _ in range(dist.get_world_size())]
            dist.all_gather(ws, w)
            same = all(torch.allclose(ws[0], t) for t in ws)
        else:
            same = True
        ckpt = None
        if ctx.get_world_rank() == 0:
            d = os.path.join(config["tmp"], f"e{epoch}")
            os.makedirs(d, exist_ok=True)
            torch.save({"epoch": epoch}, os.path.join(d, "state.pt"))
            ckpt = Checkpoint.from_directory(d)
        if config.get("fail_at") == epoch and not os.path.exists(config["marker"]):
            open(config["marker"], "w").write("x")
            raise RuntimeError("injected failure")
        train.report({"loss": loss.item(), "epoch": epoch, "synced": same,
                      "world": ctx.get_world_size()}, checkpoint=ckpt)


def test_torch_trainer_ddp_gloo(cluster, tmp_path):
    trainer = TorchTrainer(
        _loop, train_loop_config={"epochs": 4, "tmp": str(tmp_path)},
        scaling_config=ScalingConfig(num_workers=2),
        run_config=RunConfig(name="t1", storage_path=str(tmp_path / "results"),
                             checkpoint_config=CheckpointConfig(num_to_keep=2)))
    result = trainer.fit()
    assert result.metrics["epoch"] == 3
    assert result.metrics["synced"] and result.metrics["world"] == 2
    assert len(result.metrics_history) == 4
    assert result.checkpoint is not None and os.path.exists(result.checkpoint.path)
    ckpts = [d for d in os.listdir(result.path) if d.startswith("checkpoint_")]
    assert len(ckpts) == 2
    assert result.metrics_history[-1]["loss"] < result.metrics_history[0]["loss"]


def test_trainer_failure_restores_from_checkpoint(cluster, tmp_path):
    trainer = TorchTrainer(
        _loop, train_loop_config={"epochs": 4, "tmp": str(tmp_path), "fail_at": 2,
                                  "marker": str(tmp_path / "failed")},
        scaling_config=ScalingConfig(num_workers=2),
        run_config=RunConfig(name="t2", storage_path=str(tmp_path / "results"),
                             failure_config=FailureConfig(max_failures=1)))
    result = trainer.fit()
    assert result.metrics["epoch"] == 3
    epochs = [m["epoch"] for m in result.metrics_history]
    assert epochs.count(2) >= 1 and epochs[-1] == 3


def test_trainer_error_propagates(cluster, tmp_path):
    def bad(config):
        raise ValueError("boom")

    trainer = TorchTrainer(bad, scaling_config=ScalingConfig(num_workers=2),
                           run_config=RunConfig(storage_path=str(tmp_path)))
    with pytest.raises(train.TrainingFailedError):
        trainer.fit()


def test_gpt2_tiny_flat_ddp_cpu_gloo(cluster, tmp_path):
    """The headline GPT-2 step (flat buckets + fused AdamW path) across 2 gloo ranks."""

    def loop(config):
        import torch.distributed as dist

        from ray_amd.models.gpt2 import GPT2Config
        from ray_amd.train.gpt2_step import GPT2Trainer

        tr = GPT2Trainer(GPT2Config.tiny(), 2, 32, torch.device("cpu"), lr=1e-3,
                         warmup_steps=1, total_steps=10, bucket_mb=0.05)
        g = torch.Generator().manual_seed(dist.get_rank())
        x, y = tr.synthetic_batch(g)
        for i in range(3):
            loss = tr.step([(x, y)])
        p = tr.flat.p32.clone()
        ps = [torch.zeros_like(p) for _ in range(dist.get_world_size())]
        dist.all_gather(ps, p)
        train.report({"loss": float(loss), "synced": bool(torch.equal(ps[0], ps[1])),
                      "buckets": len(tr.ddp.buckets)})

    r = TorchTrainer(loop, scaling_config=ScalingConfig(num_workers=2),
                     run_config=RunConfig(storage_path=str(tmp_path))).fit()
    assert r.metrics["synced"] and r.metrics["buckets"] > 1


def _bench_json(out: str) -> dict:
    import json

    lines = [ln for ln in out.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, out[-3000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("no_ray", [False, True])
def test_bench_launcher_gloo_two_ranks(no_ray):
    """bench.py under torch.distributed.run with 2 ranks (the driver's N>1 launch), GPT-2
    tiny on gloo: the TorchTrainer path (rank 0 drives Ray, 2 Train workers) and the bare
    loop report the same world size, stay in sync and reach the same loss."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = 29600 + (7 if no_ray else 3)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--device", "cpu", "--model", "tiny", "--micro-batch", "2", "--seq-len", "64",
           "--steps", "3", "--warmup", "1"] + (["--no-ray"] if no_ray else [])
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _bench_json(r.stdout)
    assert j["n_gpus"] == 2 and j["rccl_world_size"] == 2 and j["dist_backend"] == "gloo"
    assert j["ranks_in_sync"] is True
    assert len(j["per_rank_ms_per_step"]) == 2
    assert j["config"]["launcher"] == ("torch.distributed.run (no Ray)" if no_ray
                                       else "ray_amd TorchTrainer")
    assert abs(j["final_loss"] - 6.24) < 0.05  # same seed, same synthetic data either way
    # self-diagnosing N>1 runs: per-rank exposed comm / all-reduce time, launches and
    # bytes per step (every bucket of the flat fp32 gradient once per step)
    assert j["ddp_allreduce_launches_per_step"] >= 1
    assert j["ddp_allreduce_mb_per_step"] > 0
    assert len(j["per_rank_exposed_comm_ms"]) == 2 and len(j["per_rank_allreduce_ms"]) == 2
    assert "ddp_exposed_comm_ms_per_step" in j and "ddp_bucket_busbw_gbps_mean" in j


def test_bench_allreduce_workload_gloo_two_ranks():
    """bench.py --workload allreduce: the collective size sweep (1 MiB .. 256 MiB on RCCL;
    small sizes on gloo here) with per-size time and bus bandwidth."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29621", "bench.py", "--gpus", "2",
           "--device", "cpu", "--workload", "allreduce", "--steps", "3", "--warmup", "1",
           "--max-mb", "4"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _bench_json(r.stdout)
    assert j["metric"] == "allreduce_busbw_gbps" and j["n_gpus"] == 2
    sizes = [row["mib"] for row in j["sweep"]]
    assert sizes == [1, 2, 4]
    assert all(row["busbw_gbps"] > 0 and row["ms"] > 0 for row in j["sweep"])
    assert j["value"] == j["sweep"][-1]["busbw_gbps"]


def test_accelerate_amp_bf16_and_fp16_cpu():
    """train.torch.accelerate(amp=True): prepared models autocast; fp16 adds a scaler
    behind prepare_optimizer/backward (CPU autocast path, single process)."""
    import torch

    from ray_amd.train.torch import train_loop_utils as tlu

    try:
        tlu.accelerate(amp=True)
        m = tlu.prepare_model(torch.nn.Linear(8, 4), move_to_device=False)
        y = m(torch.randn(3, 8))
        assert y.dtype == torch.bfloat16
        opt = tlu.prepare_optimizer(torch.optim.SGD(m.parameters(), lr=0.1))
        tlu.backward(y.float().sum())
        opt.step()
        assert next(m.parameters()).dtype == torch.float32
    finally:
        tlu.accelerate(amp=False)
    m2 = tlu.prepare_model(torch.nn.Linear(8, 4), move_to_device=False)
    assert m2(torch.randn(2, 8)).dtype == torch.float32


def test_accelerate_amp_keeps_state_dict_keys():
    """An AMP-prepared model has the same state_dict keys as the plain model (forward is
    patched in place, no wrapper prefix), its checkpoint loads into a plain model, and the
    patched model pickles."""
    import io

    import torch

    from ray_amd.train.torch import train_loop_utils as tlu

    def net():
        return torch.nn.Sequential(torch.nn.Linear(8, 4), torch.nn.ReLU(), torch.nn.Linear(4, 2))

    plain = tlu.prepare_model(net(), move_to_device=False)
    try:
        tlu.accelerate(amp=True)
        amp = tlu.prepare_model(net(), move_to_device=False)
    finally:
        tlu.accelerate(amp=False)
    assert list(amp.state_dict()) == list(plain.state_dict()) == list(net().state_dict())
    plain.load_state_dict(amp.state_dict())
    assert amp(torch.randn(2, 8)).dtype == torch.bfloat16
    buf = io.BytesIO()
    torch.save(amp, buf)
    buf.seek(0)
    again = torch.load(buf, weights_only=False)  # our own file
    assert again(torch.randn(2, 8)).dtype == torch.bfloat16
