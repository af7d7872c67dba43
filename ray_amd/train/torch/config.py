"""Torch backend: one process group per Train worker group on RCCL over xGMI
(reference: python/ray/train/torch/config.py).

MI355X specifics:
* backend "nccl" is RCCL on ROCm; CPU-only groups use gloo.
* all ranks on a node see the union of the group's GPUs (HIP_VISIBLE_DEVICES),
  each rank binds ``cuda:<its index in that list>`` — RCCL then uses xGMI
  peer-to-peer between the ranks' processes (the reference's
  share_cuda_visible_devices, config.py:150). Unlike the reference, the
  visibility is fixed by the raylet when it SPAWNS the worker process (the
  placement-group strategy carries ``share_gpus``), never rewritten inside a
  running actor.
* rendezvous over TCP on 127.0.0.1 for single-node groups.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from datetime import timedelta

from ray_amd.train.backend import Backend, BackendConfig


@dataclass
class TorchConfig(BackendConfig):
    backend: str | None = None
    init_method: str = "env"
    timeout_s: int = 1800

    @property
    def backend_cls(self):
        return _TorchBackend


def _check_binding():
    """Report this worker's device binding. The raylet spawned the process with
    HIP_VISIBLE_DEVICES = the union of the group's GPUs on this node and
    RAY_AMD_LOCAL_DEVICE = its own ordinal in that list (raylet._shared_visible), so
    nothing here rewrites the environment of a process that may already have
    initialised HIP."""
    return {"visible": os.environ.get("HIP_VISIBLE_DEVICES", ""),
            "local_device": int(os.environ.get("RAY_AMD_LOCAL_DEVICE", "0")),
            "gpu_ids": os.environ.get("RAY_AMD_GPU_IDS", "")}


def _init_pg(backend, master_addr, master_port, rank, world, local_rank, timeout_s):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = master_addr
    os.environ["MASTER_PORT"] = str(master_port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_RANK"] = str(local_rank)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    kw = {}
    if backend == "nccl":
        dev = int(os.environ.get("RAY_AMD_LOCAL_DEVICE", "0"))
        torch.cuda.set_device(dev)
        kw["device_id"] = torch.device("cuda", dev)
    dist.init_process_group(backend, init_method=f"tcp://{master_addr}:{master_port}",
                            rank=rank, world_size=world, timeout=timedelta(seconds=timeout_s),
                            **kw)
    return True


def _destroy_pg():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl":
            import torch

            torch.cuda.synchronize()
        dist.destroy_process_group()
    return True


class _TorchBackend(Backend):
    share_cuda_visible_devices = True

    def on_start(self, worker_group, backend_config: TorchConfig):
        import ray_amd as ray

        infos = worker_group.infos
        use_gpu = any(i["gpu_ids"] for i in infos)
        backend = backend_config.backend or ("nccl" if use_gpu else "gloo")
        if use_gpu:
            binds = ray.get([w.execute.remote(_check_binding) for w in worker_group.workers])
            seen = {}
            for b, i in zip(binds, infos):
                key = (i["node_id"], b["visible"], b["local_device"])
                if key in seen and backend == "nccl":  # RCCL: one rank per device
                    raise RuntimeError(f"two Train ranks bound to the same GPU: {b}")
                seen[key] = True
        port = ray.get(worker_group.workers[0].free_port.remote())
        local = {}
        futs = []
        for rank, (w, i) in enumerate(zip(worker_group.workers, infos)):
            lr = local.get(i["node_id"], 0)
            local[i["node_id"]] = lr + 1
            futs.append(w.execute.remote(_init_pg, backend, infos[0].get("ip", "127.0.0.1"),
                                         port, rank,
                                         len(infos), lr, backend_config.timeout_s))
        ray.get(futs)

    def on_shutdown(self, worker_group, backend_config):
        """Destroy every rank's process group (reference: train/torch/config.py:201-204
        _shutdown_torch / on_shutdown): RCCL communicators and their HIP resources are
        released before the workers are reused or stopped."""
        import ray_amd as ray

        try:
            ray.get([w.execute.remote(_destroy_pg) for w in worker_group.workers],
                    timeout=backend_config.timeout_s)
        except Exception:  # noqa: BLE001 - a dead worker has nothing left to destroy
            pass
