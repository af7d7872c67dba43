"""Option validation / resource & strategy normalisation (reference:
python/ray/_private/ray_option_utils.py)."""

from __future__ import annotations

_TASK_OPTS = {
    "num_cpus", "num_gpus", "resources", "memory", "accelerator_type", "num_returns",
    "max_retries", "retry_exceptions", "scheduling_strategy", "placement_group",
    "placement_group_bundle_index", "placement_group_capture_child_tasks", "runtime_env",
    "name", "max_calls", "object_store_memory", "_metadata", "enable_task_events", "label_selector",
    "_labels", "_generator_backpressure_num_objects",
}
_ACTOR_OPTS = {
    "num_cpus", "num_gpus", "resources", "memory", "accelerator_type", "max_concurrency",
    "max_restarts", "max_task_retries", "max_pending_calls", "name", "namespace", "lifetime",
    "scheduling_strategy", "placement_group", "placement_group_bundle_index",
    "placement_group_capture_child_tasks", "runtime_env", "concurrency_groups",
    "get_if_exists", "object_store_memory", "_metadata", "enable_task_events", "label_selector",
    "_labels",
}


def validate(opts: dict, actor: bool):
    allowed = _ACTOR_OPTS if actor else _TASK_OPTS
    for k in opts:
        if k not in allowed:
            raise ValueError(f"Invalid option keyword {k} for {'actors' if actor else 'remote functions'}.")
    for k in ("num_cpus", "num_gpus", "memory"):
        v = opts.get(k)
        if v is not None and (not isinstance(v, (int, float)) or v < 0):
            raise ValueError(f"The keyword '{k}' only accepts None or a non-negative number")
    nr = opts.get("num_returns")
    if nr is not None and not actor and not (isinstance(nr, int) and nr >= 0) and \
            nr not in ("streaming", "dynamic"):
        raise ValueError("num_returns must be a non-negative int, 'streaming' or 'dynamic'")
    res = opts.get("resources")
    if res:
        for k in ("CPU", "GPU"):
            if k in res:
                raise ValueError(f"Use the '{k.lower().replace('cpu', 'num_cpus').replace('gpu', 'num_gpus')}' "
                                 f"argument instead of resources['{k}'].")
    lt = opts.get("lifetime")
    if lt not in (None, "detached", "non_detached"):
        raise ValueError("lifetime must be 'detached', 'non_detached' or None")


def resources_of(opts: dict, actor: bool) -> dict:
    res = {}
    ncpu = opts.get("num_cpus")
    if ncpu is None:
        ncpu = 0 if actor else 1
    if ncpu:
        res["CPU"] = float(ncpu)
    ngpu = opts.get("num_gpus")
    if ngpu:
        res["GPU"] = float(ngpu)
    if opts.get("memory"):
        res["memory"] = float(opts["memory"])
    for k, v in (opts.get("resources") or {}).items():
        if v:
            res[k] = float(v)
    if opts.get("accelerator_type"):
        res[f"accelerator_type:{opts['accelerator_type']}"] = 0.001
    return res


def parse_label_selector(sel: dict) -> dict:
    """label_selector values (reference: ray.util.scheduling_strategies / label_selector):
    "v" equals, "!v" not equal, "in(a,b)" one of, "!in(a,b)" none of -> the scheduler's
    label constraint strings ("a,b" = one of, leading "!" = negated)."""
    out = {}
    for k, v in sel.items():
        if not isinstance(k, str) or not isinstance(v, str):
            raise ValueError(f"label_selector entries must be str -> str, got {k!r}: {v!r}")
        neg = v.startswith("!")
        body = v[1:] if neg else v
        if body.startswith("in(") and body.endswith(")"):
            vals = [x.strip() for x in body[3:-1].split(",") if x.strip()]
            if not vals:
                raise ValueError(f"empty in() in label_selector[{k!r}]")
            body = ",".join(vals)
        elif not body or "," in body or "(" in body:
            raise ValueError(f"invalid label_selector value {v!r} for {k!r}")
        out[k] = ("!" if neg else "") + body
    return out


def strategy_of(opts: dict):
    from ray_amd.util.placement_group import PlacementGroup
    from ray_amd.util.scheduling_strategies import (NodeAffinitySchedulingStrategy,
                                                    NodeLabelSchedulingStrategy,
                                                    PlacementGroupSchedulingStrategy)

    st = opts.get("scheduling_strategy")
    sel = opts.get("label_selector")
    if sel:
        if st not in (None, "DEFAULT"):
            raise ValueError("label_selector cannot be combined with a scheduling_strategy")
        return {"type": "node_label", "hard": parse_label_selector(sel), "soft": {}}
    pg = opts.get("placement_group")
    if pg is not None and pg != "default" and st is None:
        st = PlacementGroupSchedulingStrategy(pg, opts.get("placement_group_bundle_index", -1),
                                              opts.get("placement_group_capture_child_tasks"))
    if st is None or st == "DEFAULT":
        # inherit the parent's placement group when it captures child tasks
        from ray_amd._private import worker as W

        cw = W.global_worker.core
        if cw is not None:
            spec = getattr(cw.current_task, "spec", None) or cw.actor_spec
            if spec is not None:
                pst = spec.get("strategy")
                if isinstance(pst, dict) and pst.get("type") == "pg" and pst.get("capture"):
                    return dict(pst, bundle_index=-1)
        return None
    if st == "SPREAD":
        return "SPREAD"
    if isinstance(st, PlacementGroupSchedulingStrategy):
        p = st.placement_group
        if isinstance(p, PlacementGroup):
            out = {"type": "pg", "pg_id": p.id.hex(), "bundle_index":
                   st.placement_group_bundle_index if st.placement_group_bundle_index is not None
                   else -1, "capture": bool(st.placement_group_capture_child_tasks)}
            if getattr(st, "_share_gpus", False):
                out["share_gpus"] = True
            return out
        return None
    if isinstance(st, NodeAffinitySchedulingStrategy):
        return {"type": "node_affinity", "node_id": st.node_id, "soft": st.soft}
    if isinstance(st, NodeLabelSchedulingStrategy):
        return {"type": "node_label", "hard": st.hard, "soft": st.soft}
    if isinstance(st, dict):
        return st
    raise ValueError(f"unsupported scheduling_strategy {st!r}")
