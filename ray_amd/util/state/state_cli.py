"""``ray.util.state.state_cli`` (reference path): the ``list`` / ``get`` / ``summary``
commands of the CLI as functions (``ray_amd list actors --filter state=ALIVE`` runs
``ray_list``). The command-line wiring lives in ``ray_amd/scripts/scripts.py``."""

from __future__ import annotations

import argparse
from typing import List, Optional


def _run(fn, **kw) -> int:
    from ray_amd.scripts import scripts

    return getattr(scripts, fn)(argparse.Namespace(**kw))


def ray_list(resource: str, *, address: Optional[str] = None,
             filter: Optional[List[str]] = None, limit: int = 100,
             format: str = "table") -> int:
    return _run("cmd_list", resource=resource, address=address, filter=filter or [],
                limit=limit, format=format)


def ray_get(resource: str, id: str, *, address: Optional[str] = None) -> int:
    return _run("cmd_get", resource=resource, id=id, address=address)


def summary_state_cli(resource: str, *, address: Optional[str] = None) -> int:
    return _run("cmd_summary", resource=resource, address=address)


def task_summary(address: Optional[str] = None) -> int:
    return summary_state_cli("tasks", address=address)


def actor_summary(address: Optional[str] = None) -> int:
    return summary_state_cli("actors", address=address)


def object_summary(address: Optional[str] = None) -> int:
    return summary_state_cli("objects", address=address)
