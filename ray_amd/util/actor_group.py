"""A group of identical actors driven together (reference API: python/ray/util/actor_group.py
— ``ActorGroup(actor_cls, num_actors, num_cpus_per_actor, num_gpus_per_actor,
resources_per_actor, init_args, init_kwargs)``; ``group.method.remote(...)`` calls the method
on every member and returns the list of refs).

Members are created together and, when the cluster has room, placed by the scheduler like
any other actors; ``shutdown(patience_s)`` asks each member to exit and force-kills the ones
still alive after ``patience_s``. Optional per-member metadata comes from a
``get_actor_metadata()`` method on the class."""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any

import ray_amd as ray


@dataclass
class ActorWrapper:
    actor: Any
    metadata: Any = None


@dataclass
class ActorConfig:
    num_cpus: float = 1
    num_gpus: float = 0
    resources: dict | None = None
    init_args: tuple = ()
    init_kwargs: dict = field(default_factory=dict)


class ActorGroupMethod:
    def __init__(self, group: "ActorGroup", name: str):
        self._group = group
        self._name = name

    def __call__(self, *a, **k):
        raise TypeError(f"ActorGroup methods are invoked with .remote(): "
                        f"group.{self._name}.remote(...)")

    def remote(self, *args, **kwargs) -> list:
        return [getattr(w.actor, self._name).remote(*args, **kwargs)
                for w in self._group.actors]


class ActorGroup:
    def __init__(self, actor_cls, num_actors: int = 1, num_cpus_per_actor: float = 1,
                 num_gpus_per_actor: float = 0, resources_per_actor: dict | None = None,
                 init_args: tuple | None = None, init_kwargs: dict | None = None):
        if num_actors < 1:
            raise ValueError(f"num_actors must be positive, got {num_actors}")
        if num_cpus_per_actor < 0 or num_gpus_per_actor < 0:
            raise ValueError("CPUs and GPUs per actor must be non-negative")
        self.num_actors = num_actors
        self.actor_config = ActorConfig(num_cpus_per_actor, num_gpus_per_actor,
                                        resources_per_actor, tuple(init_args or ()),
                                        dict(init_kwargs or {}))
        opts = {"num_cpus": num_cpus_per_actor, "num_gpus": num_gpus_per_actor}
        if resources_per_actor:
            opts["resources"] = dict(resources_per_actor)
        self._cls = ray.remote(**opts)(actor_cls)
        self.actors: list[ActorWrapper] = []
        self.start()

    def __getattr__(self, name):
        if name.startswith("_") or name in ("actors", "num_actors", "actor_config"):
            raise AttributeError(name)
        if not self.actors:
            raise RuntimeError("this ActorGroup is shut down; call start() first")
        return ActorGroupMethod(self, name)

    def __len__(self):
        return len(self.actors)

    def __getitem__(self, i):
        return self.actors[i]

    def start(self):
        if self.actors:
            raise RuntimeError("the actors are already running; shutdown() first")
        self.add_actors(self.num_actors)

    def add_actors(self, n: int):
        cfg = self.actor_config
        new = [self._cls.remote(*cfg.init_args, **cfg.init_kwargs) for _ in range(n)]
        metas = [None] * n
        has_meta = [i for i, a in enumerate(new) if "get_actor_metadata" in (a._meta or {})]
        if has_meta:
            vals = ray.get([new[i].get_actor_metadata.remote() for i in has_meta])
            for i, v in zip(has_meta, vals):
                metas[i] = v
        else:
            ray.get([a.__ray_ready__.remote() for a in new])
        self.actors.extend(ActorWrapper(a, m) for a, m in zip(new, metas))

    def remove_actors(self, indexes):
        drop = set(indexes)
        self.actors = [w for i, w in enumerate(self.actors) if i not in drop]

    @property
    def actor_metadata(self):
        return [w.metadata for w in self.actors]

    def shutdown(self, patience_s: float = 5):
        if patience_s > 0 and self.actors:
            refs = [w.actor.__ray_terminate__.remote() for w in self.actors]
            _, pending = ray.wait(refs, num_returns=len(refs), timeout=patience_s)
            if pending:
                for w in self.actors:
                    ray.kill(w.actor)
        else:
            for w in self.actors:
                ray.kill(w.actor)
        self.actors = []


__all__ = ["ActorGroup", "ActorGroupMethod", "ActorWrapper", "ActorConfig"]
