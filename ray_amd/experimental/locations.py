"""``get_object_locations``: which nodes hold a copy of each object, and its size.

Reference parity: python/ray/experimental/locations.py:7. Answered from the owner's own
table (ready flag, primary-copy node, size) plus the local node's shared-memory store
listing; objects held inline by their owner (small values never enter a store) report
``node_ids == []`` like the reference's in-memory-store objects.
"""

from __future__ import annotations

import time
from typing import Any, Dict, List


def get_object_locations(obj_refs: List, timeout_ms: int = -1) -> Dict[Any, Dict[str, Any]]:
    from ray_amd._private import worker as _w
    from ray_amd.exceptions import GetTimeoutError

    if not _w.global_worker.connected:
        raise RuntimeError("Ray hasn't been initialized.")
    cw = _w._check_connected()
    deadline = None if timeout_ms is None or timeout_ms < 0 else time.monotonic() + timeout_ms / 1e3
    try:
        stored = {o["object_id"]: o for o in cw.call_raylet("list_objects")}
    except Exception:
        stored = {}
    if deadline is not None and time.monotonic() > deadline:
        raise GetTimeoutError(f"get_object_locations did not finish within {timeout_ms} ms")
    out = {}
    with cw.lock:
        for ref in obj_refs:
            oid = ref.binary()
            h = oid.hex()
            o = cw.owned.get(oid)
            s = stored.get(h)
            if o is None and s is None:
                r = cw.remote.get(oid)  # borrowed: the owner told us where the copy is
                if r is None:
                    continue  # lookup failed: excluded, like the reference
                out[ref] = {"node_ids": [r.node or cw.node_id.hex()] if r.inline is None else [],
                            "object_size": None, "device": "cpu"}
                continue
            nodes = []
            if s is not None:
                nodes.append(s["node_id"])
            elif o is not None and o.ready and o.in_store:
                nodes.append(o.node or cw.node_id.hex())
            size = s["object_size"] if s is not None else (o.size if o is not None else None)
            out[ref] = {"node_ids": nodes, "object_size": size,
                        "device": (s or {}).get("device") or "cpu"}
    return out
