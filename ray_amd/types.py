"""``ray.types`` (reference: python/ray/types.py): ``ObjectRef`` for type annotations,
e.g. ``def f(x: ObjectRef[int])``."""

from ray_amd.object_ref import ObjectRef  # noqa: F401

__all__ = ["ObjectRef"]
