"""Per-request context (reference: python/ray/serve/context.py)."""

from __future__ import annotations

import contextvars
from dataclasses import dataclass

_model_id: contextvars.ContextVar = contextvars.ContextVar("serve_model_id", default="")


@dataclass(frozen=True)
class DeploymentID:
    name: str
    app_name: str = "default"


@dataclass(frozen=True)
class ReplicaID:
    unique_id: str
    deployment_id: DeploymentID

    def to_full_id_str(self) -> str:
        return f"{self.deployment_id.app_name}#{self.deployment_id.name}#{self.unique_id}"


@dataclass
class ReplicaContext:
    """What ``serve.get_replica_context()`` returns inside a replica (also while the
    user's constructor runs)."""
    app_name: str
    deployment: str
    replica_tag: str
    servable_object: object = None

    @property
    def replica_id(self) -> ReplicaID:
        return ReplicaID(self.replica_tag.rsplit("#", 1)[-1],
                         DeploymentID(self.deployment, self.app_name))


_replica_ctx: "ReplicaContext | None" = None


def _set_replica_context(ctx):
    global _replica_ctx
    _replica_ctx = ctx


def _set_request_context(model_id):
    return _model_id.set(model_id or "")


def _reset_request_context(token):
    _model_id.reset(token)


def current_model_id():
    return _model_id.get()


def get_replica_context():
    if _replica_ctx is None:
        from ray_amd.serve.exceptions import RayServeException

        raise RayServeException("`serve.get_replica_context()` may only be called from "
                                "within a Ray Serve deployment.")
    return _replica_ctx
