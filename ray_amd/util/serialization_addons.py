"""``ray.util.serialization_addons`` (reference: python/ray/util/serialization_addons.py):
serializers for library types that need help crossing the object store."""

from __future__ import annotations


def register_starlette_serializer(serialization_context=None):
    """starlette's ``Request`` holds a receive callable and a socket scope: ship its scope
    (minus the live parts) and body-less form; the receiver gets a Request over it."""
    try:
        from starlette.requests import Request
    except ImportError:
        return
    from ray_amd.util import register_serializer

    def ser(req):
        scope = {k: v for k, v in req.scope.items() if k not in ("app", "router", "endpoint",
                                                                   "route", "state")}
        return scope

    def de(scope):
        return Request(scope)

    register_serializer(Request, serializer=ser, deserializer=de)


def register_pydantic_serializer(serialization_context=None):
    """pydantic models pickle natively in pydantic 2; nothing to register."""


def apply(serialization_context=None):
    register_pydantic_serializer(serialization_context)
    register_starlette_serializer(serialization_context)
