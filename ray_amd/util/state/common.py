"""``ray.util.state.common`` (reference: python/ray/util/state/common.py): the State API's
row types, resource names and query options.

Rows are ``StateRecord`` dicts with attribute access (``api.py``); the option dataclasses
describe a query the way the reference's do and ``StateApiClient`` accepts them."""

from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum
from typing import Any, List, Optional, Tuple, Union

from ray_amd.util.state.api import (DEFAULT_LIMIT, DEFAULT_RPC_TIMEOUT,  # noqa: F401
                                    ActorState, JobState, NodeState, ObjectState,
                                    PlacementGroupState, RuntimeEnvState, StateRecord,
                                    TaskState, WorkerState)

RAY_MAX_LIMIT_FROM_API_SERVER = 10000
DEFAULT_LOG_LIMIT = 1000

PredicateType = str  # "=" or "!="
SupportedFilterType = Union[str, bool, int, float]


class ClusterEventState(StateRecord):
    pass


class StateResource(Enum):
    ACTORS = "actors"
    JOBS = "jobs"
    PLACEMENT_GROUPS = "placement_groups"
    NODES = "nodes"
    WORKERS = "workers"
    TASKS = "tasks"
    OBJECTS = "objects"
    RUNTIME_ENVS = "runtime_envs"
    CLUSTER_EVENTS = "cluster_events"


class SummaryResource(Enum):
    ACTORS = "actors"
    TASKS = "tasks"
    OBJECTS = "objects"


RESOURCE_STATE_TYPES = {
    StateResource.ACTORS: ActorState, StateResource.JOBS: JobState,
    StateResource.PLACEMENT_GROUPS: PlacementGroupState, StateResource.NODES: NodeState,
    StateResource.WORKERS: WorkerState, StateResource.TASKS: TaskState,
    StateResource.OBJECTS: ObjectState, StateResource.RUNTIME_ENVS: RuntimeEnvState,
    StateResource.CLUSTER_EVENTS: ClusterEventState,
}


@dataclass(init=True)
class ListApiOptions:
    limit: int = DEFAULT_LIMIT
    timeout: int = DEFAULT_RPC_TIMEOUT
    detail: bool = False
    filters: Optional[List[Tuple[str, PredicateType, SupportedFilterType]]] = \
        field(default_factory=list)
    exclude_driver: bool = True
    server_timeout_multiplier: float = 0.8

    def __post_init__(self):
        if self.limit > RAY_MAX_LIMIT_FROM_API_SERVER:
            raise ValueError(f"limit {self.limit} exceeds {RAY_MAX_LIMIT_FROM_API_SERVER}")
        for f in self.filters or []:
            if len(f) != 3 or f[1] not in ("=", "!="):
                raise ValueError(f"a filter is (key, '=' | '!=', value), got {f!r}")


@dataclass(init=True)
class GetApiOptions:
    timeout: int = DEFAULT_RPC_TIMEOUT


@dataclass(init=True)
class SummaryApiOptions:
    timeout: int = DEFAULT_RPC_TIMEOUT
    filters: Optional[List[Tuple[str, PredicateType, SupportedFilterType]]] = \
        field(default_factory=list)
    summary_by: Optional[str] = None


@dataclass(init=True)
class GetLogOptions:
    timeout: int = DEFAULT_RPC_TIMEOUT
    node_id: Optional[str] = None
    node_ip: Optional[str] = None
    media_type: str = "file"
    filename: Optional[str] = None
    actor_id: Optional[str] = None
    task_id: Optional[str] = None
    attempt_number: int = 0
    pid: Optional[int] = None
    lines: int = DEFAULT_LOG_LIMIT
    interval: Optional[float] = None
    suffix: str = "out"
    submission_id: Optional[str] = None


def state_column(*, filterable: bool, detail: bool = False, format_fn=None, **kwargs) -> Any:
    """Field metadata of a state column (reference: common.state_column)."""
    return field(metadata={"filterable": filterable, "detail": detail,
                           "format_fn": format_fn}, **kwargs)
