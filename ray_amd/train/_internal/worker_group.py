"""Group of Train worker actors (reference: python/ray/train/_internal/worker_group.py)."""

from __future__ import annotations

import os
import socket
import threading
import traceback

import ray_amd as ray
from ray_amd.util.placement_group import placement_group, remove_placement_group
from ray_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy


class RayTrainWorker:
    """Actor hosting one rank of the training job."""

    def __init__(self):
        self._session = None
        self._thread = None

    def node_info(self):
        ctx = ray.get_runtime_context()
        gpu_ids = ray.get_gpu_ids()
        vis = [x for x in os.environ.get("HIP_VISIBLE_DEVICES", "").split(",") if x.strip()]
        loc = int(os.environ.get("RAY_AMD_LOCAL_DEVICE", "0"))
        # physical id of this rank's own GPU (the process may see the group's union)
        phys = [vis[loc]] if gpu_ids and loc < len(vis) else []
        return {"node_id": ctx.get_node_id(), "pid": os.getpid(),
                "gpu_ids": gpu_ids, "physical_gpu_ids": phys,
                "hostname": socket.gethostname(),
                "ip": __import__("ray_amd.util", fromlist=["x"]).get_node_ip_address()}

    def execute(self, fn, *args, **kwargs):
        return fn(*args, **kwargs)

    def free_port(self):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    def start_training(self, train_fn, config, ctx, checkpoint, shards, ckpt_index):
        from ray_amd.train._internal import session as S

        sess = S._Session(ctx, checkpoint, shards, config, ckpt_index)
        S.init_session(sess)
        self._session = sess

        def run():
            try:
                if config is None:
                    try:
                        train_fn()
                    except TypeError:
                        train_fn({})
                else:
                    train_fn(config)
                sess.results.put(("done", None, None))
            except BaseException as e:  # noqa: BLE001
                tb = traceback.format_exc()
                sess.results.put(("error", (e, tb), None))

        self._thread = threading.Thread(target=run, name="train_loop", daemon=True)
        self._thread.start()
        return True

    def get_next(self):
        """Next report from the training thread: ("report", metrics, ckpt_path) |
        ("done", ..) | ("error", (exc, tb))."""
        kind, a, b = self._session.results.get()
        if kind == "report":
            self._session.continue_ev.release()
        return kind, a, b

    def shutdown(self):
        from ray_amd.train._internal import session as S

        try:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:
            pass
        S.shutdown_session()
        return True


class WorkerGroup:
    def __init__(self, num_workers: int, resources_per_worker: dict,
                 placement_strategy: str = "PACK", actor_cls=RayTrainWorker,
                 trainer_resources: dict | None = None):
        self.num_workers = num_workers
        bundles = [dict(resources_per_worker) for _ in range(num_workers)]
        # ScalingConfig.trainer_resources: a first bundle held for the coordinator
        self._first = 1 if trainer_resources else 0
        if trainer_resources:
            bundles = [dict(trainer_resources)] + bundles
        self.pg = placement_group(bundles, strategy=placement_strategy)
        if not self.pg.wait(timeout_seconds=600):
            remove_placement_group(self.pg)
            raise RuntimeError(f"could not reserve {bundles} for the Train worker group")
        remote_cls = ray.remote(actor_cls)
        num_cpus = resources_per_worker.get("CPU", 0)
        num_gpus = resources_per_worker.get("GPU", 0)
        other = {k: v for k, v in resources_per_worker.items() if k not in ("CPU", "GPU")}
        self.workers = []
        for i in range(num_workers):
            st = PlacementGroupSchedulingStrategy(self.pg, i + self._first)
            # GPU ranks on one node see each other's devices (set at process spawn)
            st._share_gpus = bool(num_gpus)
            self.workers.append(remote_cls.options(
                num_cpus=num_cpus, num_gpus=num_gpus, resources=other or None,
                scheduling_strategy=st, max_concurrency=4).remote())
        self.infos = ray.get([w.node_info.remote() for w in self.workers])

    def execute(self, fn, *args, **kwargs):
        return ray.get([w.execute.remote(fn, *args, **kwargs) for w in self.workers])

    def execute_async(self, fn, *args, **kwargs):
        return [w.execute.remote(fn, *args, **kwargs) for w in self.workers]

    def execute_single(self, i, fn, *args, **kwargs):
        return ray.get(self.workers[i].execute.remote(fn, *args, **kwargs))

    def shutdown(self):
        try:
            ray.get([w.shutdown.remote() for w in self.workers], timeout=30)
        except Exception:
            pass
        for w in self.workers:
            try:
                ray.kill(w)
            except Exception:
                pass
        self.workers = []
        try:
            remove_placement_group(self.pg)
        except Exception:
            pass

    def __len__(self):
        return len(self.workers)
