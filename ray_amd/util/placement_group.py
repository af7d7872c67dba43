"""Placement groups (reference: python/ray/util/placement_group.py).

Bundle placement (PACK / SPREAD / STRICT_PACK / STRICT_SPREAD) runs in the native
scheduler; a committed bundle materialises `<res>_group_<pg>` resources so tasks
and actors scheduled into it are ordinary resource requests."""

from __future__ import annotations

from ray_amd._private.ids import PlacementGroupID

VALID_STRATEGIES = ("PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD")


def _cw():
    from ray_amd._private import worker as W

    return W._check_connected()


class PlacementGroup:
    def __init__(self, id: PlacementGroupID, bundle_cache=None):
        self.id = id
        self.bundle_cache = bundle_cache

    @staticmethod
    def empty():
        return PlacementGroup(PlacementGroupID.nil())

    def is_empty(self):
        return self.id.is_nil()

    def ready(self):
        """ObjectRef that resolves once the group is placed (usable in ray.get/wait)."""
        from ray_amd.remote_function import RemoteFunction

        pg = self

        def _wait_pg(pg_hex):
            from ray_amd._private import worker as W

            W.global_worker.core.call_raylet("wait_pg", pg_hex)
            return True

        global _READY_FN
        if _READY_FN is None:
            _READY_FN = RemoteFunction(_wait_pg, {"num_cpus": 0, "max_retries": 0})
        return _READY_FN.remote(pg.id.hex())

    def wait(self, timeout_seconds: float = 30) -> bool:
        from ray_amd.exceptions import GetTimeoutError

        try:
            _cw().call_raylet("wait_pg", self.id.hex(), timeout=timeout_seconds)
            return True
        except GetTimeoutError:
            return False

    @property
    def bundle_specs(self):
        if self.bundle_cache is None:
            t = _cw().call_raylet("pg_table", self.id.hex())
            self.bundle_cache = [t["bundles"][i] for i in sorted(t["bundles"])] if t else []
        return self.bundle_cache

    @property
    def bundle_count(self):
        return len(self.bundle_specs)

    def __eq__(self, o):
        return isinstance(o, PlacementGroup) and o.id == self.id

    def __hash__(self):
        return hash(self.id)

    def __repr__(self):
        return f"PlacementGroup({self.id.hex()})"


_READY_FN = None


def placement_group(bundles, strategy: str = "PACK", name: str = "", lifetime=None,
                    _max_cpu_fraction_per_node=None, _soft_target_node_id=None) -> PlacementGroup:
    if not isinstance(bundles, list) or not bundles:
        raise ValueError("The placement group `bundles` argument cannot contain an empty list")
    for b in bundles:
        if not isinstance(b, dict) or not b:
            raise ValueError("Bundles cannot be an empty dictionary or a non-dict: "
                             f"bundles={bundles}")
        if all(v == 0 for v in b.values()):
            raise ValueError(f"Bundles cannot contain only zero resources: {b}")
        for v in b.values():
            if v < 0:
                raise ValueError("bundle resources must be non-negative")
    if strategy not in VALID_STRATEGIES:
        raise ValueError(f"Invalid placement group strategy {strategy}. Supported strategies "
                         f"are: {VALID_STRATEGIES}.")
    if _max_cpu_fraction_per_node is not None or _soft_target_node_id is not None:
        # experimental reference knobs (deprecated there): refused rather than ignored
        raise NotImplementedError("_max_cpu_fraction_per_node / _soft_target_node_id are not "
                                  "supported by this scheduler")
    if lifetime not in (None, "detached"):
        raise ValueError("placement group `lifetime` argument must be either `None` or "
                         "'detached'")
    cw = _cw()
    pgid = PlacementGroupID.from_random()
    cw.call_raylet("create_pg", pgid.hex(), [dict(b) for b in bundles], strategy, name or None,
                   lifetime, cw.addr, cw.namespace)
    return PlacementGroup(pgid, [dict(b) for b in bundles])


def remove_placement_group(placement_group: PlacementGroup):
    _cw().call_raylet("remove_pg", placement_group.id.hex())


def get_placement_group(placement_group_name: str) -> PlacementGroup:
    cw = _cw()
    info = cw.call_raylet("get_named_pg", placement_group_name, cw.namespace)
    if info is None:
        raise ValueError(f"Failed to look up placement group with name: {placement_group_name}")
    return PlacementGroup(PlacementGroupID.from_hex(info["pg_id"]), info["bundles"])


def placement_group_table(placement_group: PlacementGroup | None = None) -> dict:
    cw = _cw()
    return cw.call_raylet("pg_table", placement_group.id.hex() if placement_group else None)


def get_current_placement_group() -> PlacementGroup | None:
    from ray_amd._private import worker as W

    cw = W.global_worker.core
    if cw is None:
        return None
    # a task's own strategy, else (actor method calls carry none) the actor's creation one
    for spec in (getattr(cw.current_task, "spec", None), cw.actor_spec):
        st = spec.get("strategy") if spec else None
        if isinstance(st, dict) and st.get("type") == "pg":
            return PlacementGroup(PlacementGroupID.from_hex(st["pg_id"]))
    return None


def check_placement_group_index(placement_group, bundle_index):
    if bundle_index < -1 or (placement_group is not None and bundle_index >=
                             placement_group.bundle_count):
        raise ValueError("placement_group_bundle_index out of range")
