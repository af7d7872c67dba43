"""``ray.util.serialization`` (reference: python/ray/util/serialization.py): custom
serializers for types cloudpickle cannot handle, registered per process."""

from ray_amd._private.serialization import (deregister_serializer,  # noqa: F401
                                            register_serializer)

__all__ = ["register_serializer", "deregister_serializer"]
