"""``ray.util.check_serialize`` (reference: python/ray/util/check_serialize.py): find the
members of an object that make it unpicklable."""

from ray_amd.util import inspect_serializability  # noqa: F401

__all__ = ["inspect_serializability"]
