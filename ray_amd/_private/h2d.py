"""Pinned H2D from the shared-memory object store.

A numpy view of an object in the /dev/shm store is pageable memory to HIP: ``.to("cuda")``
then copies through the runtime's bounce buffers. Registering the store pages with
``hipHostRegister`` makes the same copy a direct DMA (``torch`` sees the pointer as pinned
and issues an async copy). The store can be hundreds of GB, so it is never registered as a
whole: ``StorePinCache`` registers the fixed 64 MiB chunks that a copy touches, keeps them
registered (blocks are recycled through the same heap regions by the streaming executor)
and unregisters the least recently used chunks beyond a byte cap.

The copy is asynchronous, so two things must outlive it: the chunk registration (an
unregister under an in-flight DMA would fault or fall back mid-copy) and the store object
the numpy view points into (a released block is recycled by the next ``put``). Every copy
records a HIP event; the chunks it touched remember that event and an eviction waits on it
first, and the source array is held in a pending list until its event has completed.

Enabled in the Ray Data GPU preprocessing actors with ``RAY_AMD_DATA_PIN_STORE=1``
(reference config 4, "pinned async H2D"; ``ray_amd/data/preprocessors.py``).
"""

from __future__ import annotations

import collections
import os
import threading

CHUNK = 64 << 20


class StorePinCache:
    def __init__(self, base: int, size: int, cap_bytes: int, lib=None):
        self.base, self.size, self.cap = base, size, cap_bytes
        self._lib = lib
        self._chunks = collections.OrderedDict()  # chunk index -> True (LRU order)
        self._lock = threading.Lock()
        self.registered_bytes = 0
        self.failures = 0
        self._last_use = {}  # chunk index -> event of the latest copy that read it
        self._pending = collections.deque()  # (event, source array) of in-flight copies

    def _L(self):
        if self._lib is None:
            from ray_amd.ops import _lib

            self._lib = _lib.lib()
        return self._lib

    def covers(self, ptr: int, n: int) -> bool:
        return self.base <= ptr and ptr + n <= self.base + self.size

    def ensure(self, ptr: int, n: int) -> bool:
        """Register every chunk of [ptr, ptr + n); False when the range is outside the store
        or a registration failed (the copy then simply runs pageable)."""
        if n <= 0 or not self.covers(ptr, n):
            return False
        first = (ptr - self.base) // CHUNK
        last = (ptr + n - 1 - self.base) // CHUNK
        with self._lock:
            ok = True
            for c in range(first, last + 1):
                if c in self._chunks:
                    self._chunks.move_to_end(c)
                    continue
                start = self.base + c * CHUNK
                length = min(CHUNK, self.base + self.size - start)
                if self._L().ra_host_register(start, length) != 0:
                    self.failures += 1
                    ok = False
                    continue
                self._chunks[c] = length
                self.registered_bytes += length
            while self.registered_bytes > self.cap and len(self._chunks) > last - first + 1:
                c, length = self._chunks.popitem(last=False)
                if first <= c <= last:  # never drop a chunk this copy needs
                    self._chunks[c] = length
                    self._chunks.move_to_end(c, last=False)
                    break
                ev = self._last_use.pop(c, None)
                if ev is not None:
                    ev.synchronize()  # a copy still reading this chunk finishes first
                self._L().ra_host_unregister(self.base + c * CHUNK)
                self.registered_bytes -= length
            return ok

    def track(self, ptr: int, n: int, event, src) -> None:
        """Record that an async copy of [ptr, ptr + n) completes at ``event``: the chunks it
        read stay registered and ``src`` stays referenced until then."""
        with self._lock:
            if n > 0 and self.covers(ptr, n):
                for c in range((ptr - self.base) // CHUNK,
                               (ptr + n - 1 - self.base) // CHUNK + 1):
                    if c in self._chunks:
                        self._last_use[c] = event
            self._pending.append((event, src))
            while self._pending and self._pending[0][0].query():
                self._pending.popleft()

    def drain(self) -> None:
        """Wait for every tracked copy (tests, shutdown)."""
        with self._lock:
            while self._pending:
                self._pending.popleft()[0].synchronize()
            self._last_use.clear()


_cache = None
_cache_lock = threading.Lock()


def store_pin_cache():
    """This process's cache over its object-store mapping (None outside a worker)."""
    global _cache
    if _cache is not None:
        return _cache
    with _cache_lock:
        if _cache is None:
            from ray_amd._private.worker import global_worker

            cw = global_worker.core
            if cw is None or getattr(cw, "store", None) is None:
                return None
            st = cw.store.store
            cap = int(float(os.environ.get("RAY_AMD_PIN_STORE_CAP_GB", "8")) * (1 << 30))
            _cache = StorePinCache(int(st.address()), int(st.size), cap)
    return _cache


def to_device_pinned(arr, device):
    """``torch.from_numpy(arr).to(device)`` with the store pages behind ``arr`` registered
    first (when ``arr`` is a view into the object store)."""
    import torch

    t = torch.from_numpy(arr)
    c = store_pin_cache()
    ptr = arr.__array_interface__["data"][0]
    if c is None or not c.ensure(ptr, arr.nbytes):
        return t.to(device)  # pageable: the runtime stages it and the call returns done
    out = t.to(device, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(out.device))
    c.track(ptr, arr.nbytes, ev, arr)
    return out
