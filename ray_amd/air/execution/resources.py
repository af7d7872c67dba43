"""Resource requests and managers (reference: python/ray/air/execution/resources/
request.py:32, fixed.py:43, placement_group.py:46).

A ``ResourceRequest`` is a list of bundles plus a placement strategy; the first bundle is
the "head" (e.g. a Tune trial's trainable), the rest serve workers it starts. A
``ResourceManager`` turns requests into ``AcquiredResources``:

* ``PlacementGroupResourceManager`` reserves one placement group per request (the native
  bundle scheduler places it), reports it ready when the group is placed, and hands out
  ``PlacementGroupAcquiredResources`` whose ``annotate_remote_entities`` pins remote
  functions / actor classes to the group's bundles;
* ``FixedResourceManager`` does bookkeeping against a fixed resource total without
  touching the cluster (for controllers running inside a job that already holds its
  resources).
"""

from __future__ import annotations

import time
from typing import Dict, List, Optional


def _sum_bundles(bundles):
    out: Dict[str, float] = {}
    for b in bundles:
        for k, v in b.items():
            out[k] = out.get(k, 0.0) + v
    return out


class ResourceRequest:
    def __init__(self, bundles: List[Dict[str, float]], strategy: str = "PACK",
                 *args, **kwargs):
        if not bundles:
            raise ValueError("a ResourceRequest needs at least one bundle")
        self._head_empty = not any(v for v in bundles[0].values())
        self._bundles = [{k: v for k, v in b.items() if v} for b in bundles]
        if self._head_empty:
            self._bundles = self._bundles[1:] or [{}]
        if strategy not in ("PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD"):
            raise ValueError(f"invalid placement strategy {strategy!r}")
        self._strategy = strategy
        self._args, self._kwargs = args, kwargs

    @property
    def head_bundle_is_empty(self) -> bool:
        return self._head_empty

    @property
    def head_cpus(self) -> float:
        return 0.0 if self._head_empty else self._bundles[0].get("CPU", 0.0)

    @property
    def bundles(self) -> List[Dict[str, float]]:
        return [dict(b) for b in self._bundles]

    @property
    def required_resources(self) -> Dict[str, float]:
        return _sum_bundles(self._bundles)

    @property
    def strategy(self) -> str:
        return self._strategy

    def to_placement_group(self):
        from ray_amd.util.placement_group import placement_group

        return placement_group(self.bundles, strategy=self._strategy, *self._args,
                               **self._kwargs)

    def _key(self):
        return (self._head_empty, tuple(tuple(sorted(b.items())) for b in self._bundles),
                self._strategy)

    def __eq__(self, other):
        return isinstance(other, ResourceRequest) and self._key() == other._key()

    def __hash__(self):
        return hash(self._key())

    def __repr__(self):
        return (f"<ResourceRequest (_bound={self._head_empty}): bundles={self._bundles} "
                f"strategy={self._strategy}>")


class AcquiredResources:
    def __init__(self, resource_request: ResourceRequest):
        self.resource_request = resource_request

    def annotate_remote_entities(self, entities: list) -> list:
        """One entity (remote function / actor class) per bundle, in bundle order; the
        head bundle's entity comes first unless the head bundle was empty."""
        bundles = self.resource_request.bundles
        if len(entities) > len(bundles):
            raise RuntimeError(f"{len(entities)} entities for {len(bundles)} bundles")
        return [self._annotate(e, bundles[i], i) for i, e in enumerate(entities)]

    def _annotate(self, entity, bundle, index):
        raise NotImplementedError


def _resource_opts(bundle: dict) -> dict:
    opts = {"num_cpus": bundle.get("CPU", 0), "num_gpus": bundle.get("GPU", 0)}
    other = {k: v for k, v in bundle.items() if k not in ("CPU", "GPU", "memory")}
    if other:
        opts["resources"] = other
    if bundle.get("memory"):
        opts["memory"] = bundle["memory"]
    return opts


class FixedAcquiredResources(AcquiredResources):
    def _annotate(self, entity, bundle, index):
        return entity.options(**_resource_opts(bundle))


class PlacementGroupAcquiredResources(AcquiredResources):
    def __init__(self, resource_request, placement_group):
        super().__init__(resource_request)
        self.placement_group = placement_group

    def _annotate(self, entity, bundle, index):
        from ray_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy

        return entity.options(
            scheduling_strategy=PlacementGroupSchedulingStrategy(
                self.placement_group, placement_group_bundle_index=index),
            **_resource_opts(bundle))


class ResourceManager:
    def request_resources(self, resource_request: ResourceRequest):
        raise NotImplementedError

    def cancel_resource_request(self, resource_request: ResourceRequest):
        raise NotImplementedError

    def has_resources_ready(self, resource_request: ResourceRequest) -> bool:
        raise NotImplementedError

    def acquire_resources(self, resource_request: ResourceRequest
                          ) -> Optional[AcquiredResources]:
        raise NotImplementedError

    def free_resources(self, acquired_resource: AcquiredResources):
        raise NotImplementedError

    def get_resource_futures(self) -> list:
        return []

    def update_state(self):
        pass

    def clear(self):
        raise NotImplementedError

    def __reduce__(self):
        raise ValueError("Resource managers cannot be serialized")


class FixedResourceManager(ResourceManager):
    def __init__(self, total_resources: Optional[Dict[str, float]] = None):
        if total_resources is None:
            import ray_amd as ray

            total_resources = dict(ray.available_resources()) if ray.is_initialized() \
                else {}
        self._total = dict(total_resources)
        self._used: Dict[str, float] = {}
        self._requested: list = []
        self._acquired: list = []

    def _available(self):
        return {k: v - self._used.get(k, 0.0) for k, v in self._total.items()}

    def request_resources(self, resource_request):
        self._requested.append(resource_request)

    def cancel_resource_request(self, resource_request):
        self._requested.remove(resource_request)

    def has_resources_ready(self, resource_request):
        if resource_request not in self._requested:
            return False
        avail = self._available()
        return all(avail.get(k, 0.0) >= v - 1e-9
                   for k, v in resource_request.required_resources.items())

    def acquire_resources(self, resource_request):
        if not self.has_resources_ready(resource_request):
            return None
        self._requested.remove(resource_request)
        for k, v in resource_request.required_resources.items():
            self._used[k] = self._used.get(k, 0.0) + v
        acq = FixedAcquiredResources(resource_request)
        self._acquired.append(acq)
        return acq

    def free_resources(self, acquired_resource):
        self._acquired.remove(acquired_resource)
        for k, v in acquired_resource.resource_request.required_resources.items():
            self._used[k] -= v

    def clear(self):
        self._requested.clear()
        self._acquired.clear()
        self._used.clear()


class PlacementGroupResourceManager(ResourceManager):
    def __init__(self, update_interval_s: float = 0.1):
        self.update_interval_s = update_interval_s
        self._pending: Dict[ResourceRequest, list] = {}  # request -> [placement groups]
        self._ready: Dict[ResourceRequest, list] = {}
        self._acquired: list = []
        self._last = 0.0

    def request_resources(self, resource_request):
        pg = resource_request.to_placement_group()
        self._pending.setdefault(resource_request, []).append(pg)

    def cancel_resource_request(self, resource_request):
        from ray_amd.util.placement_group import remove_placement_group

        for table in (self._pending, self._ready):
            pgs = table.get(resource_request)
            if pgs:
                remove_placement_group(pgs.pop())
                if not pgs:
                    del table[resource_request]
                return

    @staticmethod
    def _placed(pg) -> bool:
        from ray_amd.util.placement_group import placement_group_table

        return (placement_group_table(pg) or {}).get("state") == "CREATED"

    def update_state(self):
        for req, pgs in list(self._pending.items()):
            for pg in list(pgs):
                if self._placed(pg):
                    pgs.remove(pg)
                    self._ready.setdefault(req, []).append(pg)
            if not pgs:
                del self._pending[req]
        self._last = time.monotonic()

    def _maybe_update(self):
        if time.monotonic() - self._last >= self.update_interval_s:
            self.update_state()

    def get_resource_futures(self) -> list:
        return [pg.ready() for pgs in self._pending.values() for pg in pgs]

    def has_resources_ready(self, resource_request):
        self._maybe_update()
        return bool(self._ready.get(resource_request))

    def acquire_resources(self, resource_request):
        if not self.has_resources_ready(resource_request):
            return None
        pg = self._ready[resource_request].pop(0)
        if not self._ready[resource_request]:
            del self._ready[resource_request]
        acq = PlacementGroupAcquiredResources(resource_request, pg)
        self._acquired.append(acq)
        return acq

    def free_resources(self, acquired_resource):
        from ray_amd.util.placement_group import remove_placement_group

        self._acquired.remove(acquired_resource)
        remove_placement_group(acquired_resource.placement_group)

    def clear(self):
        from ray_amd.util.placement_group import remove_placement_group

        for table in (self._pending, self._ready):
            for pgs in table.values():
                for pg in pgs:
                    remove_placement_group(pg)
            table.clear()
        for acq in self._acquired:
            remove_placement_group(acq.placement_group)
        self._acquired.clear()
