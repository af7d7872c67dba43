"""Cluster KV store (reference: python/ray/experimental/internal_kv.py)."""

from __future__ import annotations


def _cw():
    from ray_amd._private import worker as W

    return W._check_connected()


def _ns(namespace):
    return "kv:" + (namespace.decode() if isinstance(namespace, bytes) else (namespace or ""))


def _internal_kv_initialized():
    from ray_amd._private import worker as W

    return W.global_worker.connected


def _internal_kv_put(key, value, overwrite: bool = True, namespace=None) -> bool:
    """Returns True if the key already existed."""
    if isinstance(value, str):
        value = value.encode()
    added = _cw().call_raylet("kv_put", _ns(namespace), key, value, overwrite)
    return not added


def _internal_kv_get(key, namespace=None):
    return _cw().call_raylet("kv_get", _ns(namespace), key)


def _internal_kv_exists(key, namespace=None) -> bool:
    return _cw().call_raylet("kv_exists", _ns(namespace), key)


def _internal_kv_del(key, del_by_prefix: bool = False, namespace=None) -> int:
    return _cw().call_raylet("kv_del", _ns(namespace), key, del_by_prefix)


def _internal_kv_list(prefix, namespace=None):
    return _cw().call_raylet("kv_keys", _ns(namespace), prefix)
