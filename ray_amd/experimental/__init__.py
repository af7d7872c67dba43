"""Experimental APIs (reference: python/ray/experimental/__init__.py)."""

from ray_amd.experimental.locations import get_object_locations  # noqa: F401
from ray_amd.experimental.packaging.load_package import load_package  # noqa: F401


def set_resource(resource_name, capacity, node_id=None):
    """Dynamic custom resources were removed upstream; the reference raises the same."""
    raise DeprecationWarning(
        "Dynamic custom resources are deprecated. Consider using placement groups "
        "instead, or specify resources when the node starts (the 'resources' field).")


__all__ = ["get_object_locations", "set_resource", "load_package"]
