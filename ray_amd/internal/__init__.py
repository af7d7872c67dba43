"""Low-level internal API (reference: python/ray/internal/__init__.py ->
python/ray/_private/internal_api.py:177 ``free``)."""

from __future__ import annotations

__all__ = ["free"]


def free(object_refs: list, local_only: bool = False) -> None:
    """Free the stored values of ``object_refs`` now, whatever their reference counts.

    An instruction to the object stores, with no return value: a later ``get`` of a freed
    object raises ``ObjectFreedError`` and the object is never reconstructed from lineage.
    ``local_only=True`` only drops this node's store copy of objects owned elsewhere."""
    from ray_amd._private import worker as W
    from ray_amd.object_ref import ObjectRef

    if isinstance(object_refs, ObjectRef):
        object_refs = [object_refs]
    if not isinstance(object_refs, list):
        raise TypeError(f"free() expects a list of ObjectRef, got {type(object_refs)}")
    for r in object_refs:
        if not isinstance(r, ObjectRef):
            raise TypeError(f"Attempting to call `free` on the value {r!r}, which is not an "
                            "ObjectRef.")
    core = W.global_worker.core
    if core is None:
        raise RuntimeError("ray_amd.init() must be called first")
    if object_refs:
        core.free_objects([r._id for r in object_refs], local_only)
