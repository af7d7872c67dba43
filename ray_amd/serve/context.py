"""Per-request context (reference: python/ray/serve/context.py)."""

from __future__ import annotations

import contextvars
from dataclasses import dataclass

_model_id: contextvars.ContextVar = contextvars.ContextVar("serve_model_id", default="")


@dataclass
class ReplicaContext:
    app_name: str
    deployment: str
    replica_tag: str


def _set_request_context(model_id):
    return _model_id.set(model_id or "")


def _reset_request_context(token):
    _model_id.reset(token)


def current_model_id():
    return _model_id.get()


def get_replica_context():
    return None
