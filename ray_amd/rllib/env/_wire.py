"""JSON wire format of the external-env client/server (numpy arrays as typed lists)."""

from __future__ import annotations

import json

import numpy as np


def _enc(x):
    if isinstance(x, np.ndarray):
        return {"__nd__": x.tolist(), "dtype": str(x.dtype), "shape": list(x.shape)}
    if isinstance(x, np.generic):
        return x.item()
    if isinstance(x, dict):
        return {"__map__": [[_enc(k), _enc(v)] for k, v in x.items()]}
    if isinstance(x, (list, tuple)):
        return [_enc(v) for v in x]
    return x


def _dec(x):
    if isinstance(x, dict):
        if "__nd__" in x:
            return np.asarray(x["__nd__"], dtype=x["dtype"]).reshape(x["shape"])
        if "__map__" in x:
            return {_key(_dec(k)): _dec(v) for k, v in x["__map__"]}
        return {k: _dec(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_dec(v) for v in x]
    return x


def _key(k):
    return tuple(k) if isinstance(k, list) else k


def dumps(obj) -> bytes:
    return json.dumps(_enc(obj)).encode()


def loads(b: bytes):
    return _dec(json.loads(b.decode()))
