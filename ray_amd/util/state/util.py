"""``ray.util.state.util`` (reference: python/ray/util/state/util.py)."""

from __future__ import annotations

from typing import Union


def convert_string_to_type(val: Union[str, int, float, bool], convert_type):
    """A filter value given as text, as the column's type."""
    if convert_type is int:
        return int(val)
    if convert_type is float:
        return float(val)
    if convert_type is bool:
        if isinstance(val, bool):
            return val
        low = str(val).lower()
        if low in ("true", "1"):
            return True
        if low in ("false", "0"):
            return False
        raise ValueError(f"expected a boolean, got {val!r}")
    return val


def record_deprecated_state_api_import():
    """The reference logs a usage tag here; nothing to record in ray_amd."""
