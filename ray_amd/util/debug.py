"""``log_once`` rate limiting for warnings (reference: python/ray/util/debug.py:17-67)."""

from __future__ import annotations

import threading
import time

_logged: set = set()
_disabled = False
_periodic_until = 0.0
_lock = threading.Lock()


def log_once(key) -> bool:
    """True the first time `key` is seen (and always while periodic logging is enabled)."""
    global _periodic_until
    with _lock:
        if _disabled:
            return False
        if time.monotonic() < _periodic_until:
            return True
        if key in _logged:
            return False
        _logged.add(key)
        return True


def disable_log_once_globally():
    global _disabled
    _disabled = True


def enable_periodic_logging(period_s: float = 60.0):
    """log_once returns True for every key during the next `period_s` seconds."""
    global _periodic_until
    _periodic_until = time.monotonic() + period_s


def reset_log_once(key=None):
    with _lock:
        if key is None:
            _logged.clear()
        else:
            _logged.discard(key)
