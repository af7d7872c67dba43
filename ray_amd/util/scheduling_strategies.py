"""Scheduling strategies (reference: python/ray/util/scheduling_strategies.py)."""

from __future__ import annotations


class PlacementGroupSchedulingStrategy:
    def __init__(self, placement_group, placement_group_bundle_index: int = -1,
                 placement_group_capture_child_tasks: bool | None = None):
        self.placement_group = placement_group
        self.placement_group_bundle_index = placement_group_bundle_index
        self.placement_group_capture_child_tasks = placement_group_capture_child_tasks


class NodeAffinitySchedulingStrategy:
    def __init__(self, node_id: str, soft: bool, _spill_on_unavailable: bool = False,
                 _fail_on_unavailable: bool = False):
        self.node_id = node_id if isinstance(node_id, str) else node_id.hex()
        self.soft = soft
        self._spill_on_unavailable = _spill_on_unavailable
        self._fail_on_unavailable = _fail_on_unavailable


class In:
    def __init__(self, *values):
        self.values = list(values)


class NotIn:
    def __init__(self, *values):
        self.values = list(values)


class Exists:
    pass


class DoesNotExist:
    pass


class NodeLabelSchedulingStrategy:
    def __init__(self, hard: dict, *, soft: dict | None = None):
        self.hard = {k: (v.values if isinstance(v, In) else v) for k, v in (hard or {}).items()}
        self.soft = {k: (v.values if isinstance(v, In) else v) for k, v in (soft or {}).items()}


SchedulingStrategyT = object
DEFAULT_SCHEDULING_STRATEGY = "DEFAULT"
SPREAD_SCHEDULING_STRATEGY = "SPREAD"
