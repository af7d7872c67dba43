"""``ray.serve.grpc_util`` (reference: python/ray/serve/grpc_util.py): a picklable snapshot
of a gRPC servicer context that a deployment can read and annotate (code, details,
trailing metadata) and the proxy applies to the reply."""

from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple


class RayServegRPCContext:
    def __init__(self, grpc_context=None):
        g = grpc_context
        self._auth_context = _call(g, "auth_context", {}) or {}
        self._code = _call(g, "code", None)
        self._details = _call(g, "details", None)
        self._invocation_metadata = [(k, v) for k, v in (_call(g, "invocation_metadata", ())
                                                         or ())]
        self._peer = _call(g, "peer", None)
        self._peer_identities = _call(g, "peer_identities", None)
        self._peer_identity_key = _call(g, "peer_identity_key", None)
        self._trailing_metadata = [(k, v) for k, v in (_call(g, "trailing_metadata", ())
                                                       or ())]
        self._compression = None

    def auth_context(self) -> Dict[str, Any]:
        return self._auth_context

    def code(self):
        return self._code

    def details(self) -> Optional[str]:
        return self._details

    def invocation_metadata(self) -> List[Tuple[str, str]]:
        return self._invocation_metadata

    def peer(self) -> Optional[str]:
        return self._peer

    def peer_identities(self):
        return self._peer_identities

    def peer_identity_key(self):
        return self._peer_identity_key

    def trailing_metadata(self) -> List[Tuple[str, str]]:
        return self._trailing_metadata

    def set_code(self, code):
        self._code = code

    def set_compression(self, compression):
        self._compression = compression

    def set_details(self, details: str):
        self._details = details

    def set_trailing_metadata(self, trailing_metadata: List[Tuple[str, str]]):
        self._trailing_metadata = list(trailing_metadata)

    def _set_on_grpc_context(self, grpc_context):
        """Copy what the deployment set onto the live servicer context (proxy side)."""
        if self._code is not None:
            grpc_context.set_code(self._code)
        if self._details:
            grpc_context.set_details(self._details)
        if self._trailing_metadata:
            grpc_context.set_trailing_metadata(tuple(self._trailing_metadata))
        if self._compression is not None:
            grpc_context.set_compression(self._compression)


def _call(obj, name, default):
    f = getattr(obj, name, None)
    if f is None:
        return default
    try:
        return f()
    except Exception:  # noqa: BLE001 - not every context implements every accessor
        return default
