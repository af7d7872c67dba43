"""Node-local object store client (reference: plasma client + external_storage.py spilling).

Wraps the native ``_core.ShmStore``: every process on the node maps the same
/dev/shm segment, so put/get are in-process operations (no store IPC).
When the heap is full: evict unpinned secondary copies (LRU), then spill pinned
primary copies to ``<session>/spill/<oid>`` (write + rename, THEN drop from the
store, so a concurrent reader that misses the store always finds the file).
Spilled objects are read back through mmap — still zero-copy.
"""

from __future__ import annotations

import mmap
import os
import threading

from ray_amd._native import _core
from ray_amd.exceptions import ObjectStoreFullError

from . import serialization as ser

NO_SPACE = (1 << 64) - 1
# writes at least this large map their destination pages with one madvise first
# (ShmStore.populate): per-page write faults cost more than the copy itself
POPULATE_MIN = 1 << 20


def table_capacity(store_bytes: int) -> int:
    """Object-table slots for a store of ``store_bytes``: one per 16 KiB (small objects
    live inline in their owner's memory store, not here), between 4096 and 2^18."""
    return max(4096, min(1 << 18, int(store_bytes) >> 14))


def start_prefault(store, size: int):
    """Back the low end of a freshly created store's heap with pages in a daemon thread
    (ShmStore.populate(write=True): allocates + zeroes holes, never touches data), so
    writers' populate-read finds pages already allocated. RAY_AMD_STORE_PREFAULT_BYTES
    (default: the smallest of a quarter of the store, 1/64 of RAM and 4 GiB; 0 disables).
    Measured on the MI355X box: 16 workers faulting fresh pages of the same segment at
    once take ~80 ms per 36 MiB block (allocation contention) against ~2 ms for pages
    already backed."""
    try:
        ram = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES")
    except (ValueError, OSError):
        ram = 64 << 30
    n = int(os.environ.get("RAY_AMD_STORE_PREFAULT_BYTES", min(size // 4, ram // 64, 4 << 30)))
    if n <= 0:
        return None
    base = store.heap_offset
    stop = threading.Event()

    def run():
        chunk = 32 << 20
        for off in range(base, base + n, chunk):
            if stop.is_set() or not store.populate(off, min(chunk, base + n - off), True):
                return

    t = threading.Thread(target=run, name="store-prefault", daemon=True)
    t.start()

    def finish():
        # a daemon thread still inside the native call (GIL released) when the
        # interpreter finalises is unwound through noexcept C++ frames: std::terminate
        stop.set()
        t.join()

    import atexit

    atexit.register(finish)
    return t


class _MmapBuf:
    """Keeps a spill-file mapping alive while views of it exist."""

    __slots__ = ("mm", "mv")

    def __init__(self, path):
        with open(path, "rb") as f:
            self.mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
        self.mv = memoryview(self.mm)


class ObjectStore:
    def __init__(self, path: str, spill_dir: str, create: bool = False, size: int = 0,
                 table_cap: int = 1 << 18):
        self.path = path
        self.spill_dir = spill_dir
        self.store = _core.ShmStore(path, size, create, table_cap)
        os.makedirs(spill_dir, exist_ok=True)
        self._lock = threading.Lock()
        self.spilled_bytes = 0
        self.restored_bytes = 0
        self.fallback_bytes = 0
        self.fallback_objects = 0
        self.waited_allocs = 0

    # ------------------------------------------------------------------ write
    def _try_make_room(self, oid: bytes, size: int, pinned: bool, device: int) -> int:
        off = self.store.create(oid, size, 0, device, pinned)
        if off != NO_SPACE:
            return off
        # 1) evict unpinned LRU copies
        self.store.evict(size * 2, device)
        off = self.store.create(oid, size, 0, device, pinned)
        if off != NO_SPACE or device >= 0:
            return off
        # 2) spill pinned primary copies
        for _ in range(8):
            cands = self.store.spill_candidates(max(size * 2, 64 << 20), device)
            if not cands:
                break
            for c in cands:
                self.spill(c)
            off = self.store.create(oid, size, 0, device, pinned)
            if off != NO_SPACE:
                return off
        return NO_SPACE

    def _spill_pending(self) -> bool:
        """Another process on the node is writing a spill file right now (its space frees
        when the write completes: ``spill`` writes ``<oid>.tmp<pid>`` then renames)."""
        try:
            with os.scandir(self.spill_dir) as it:
                return any(".tmp" in e.name for e in it)
        except FileNotFoundError:
            return False

    def _alloc(self, oid: bytes, size: int, pinned: bool, device: int = -1, wait: bool = True):
        """Offset of a new ``size``-byte entry, or None: the caller then writes the object
        to the disk-backed fallback (``_fallback_write``).

        The create-request queue of plasma (reference: src/ray/object_manager/plasma/
        create_request_queue.cc:89-125, plasma_allocator.cc:62-70), per request: evict,
        spill, and if the object still does not fit, WAIT — with exponential backoff, a
        local gc pass that drops unreachable zero-copy readers, and the wait extended
        for as long as spills are in flight — up to ``oom_grace_period_s``
        (RAY_AMD_OOM_GRACE_PERIOD_S, default 2 s as the reference) of no progress; then
        allocate from the fallback (a file under the session's spill directory, read
        back zero-copy through mmap and deleted with the object)."""
        off = self._try_make_room(oid, size, pinned, device)
        if off != NO_SPACE:
            return off
        if device >= 0:
            raise ObjectStoreFullError(f"HBM object store on GPU {device} is full "
                                       f"({self.store.used(device)} / "
                                       f"{self.store.capacity(device)} bytes)")
        if not wait:
            return None
        if size > self.store.capacity(-1) or os.environ.get("RAY_AMD_OBJECT_STORE_FALLBACK",
                                                             "1") == "0":
            if os.environ.get("RAY_AMD_OBJECT_STORE_FALLBACK", "1") == "0":
                raise ObjectStoreFullError(
                    f"object of {size} bytes does not fit in the object store "
                    f"({self.store.used(-1)} / {self.store.capacity(-1)} bytes in use, "
                    "nothing spillable)")
            return None  # larger than the whole store: straight to the fallback
        import gc
        import time

        grace = float(os.environ.get("RAY_AMD_OOM_GRACE_PERIOD_S", "2.0"))
        delay = float(os.environ.get("RAY_AMD_OBJECT_STORE_FULL_DELAY_MS", "10")) / 1000.0
        start = time.monotonic()
        gc_done = False
        while True:
            if not gc_done:
                gc.collect()  # reference: trigger_global_gc_ (this process's share)
                gc_done = True
            time.sleep(delay)
            delay = min(delay * 2, 0.1)
            off = self._try_make_room(oid, size, pinned, device)
            if off != NO_SPACE:
                self.waited_allocs += 1
                return off
            if self._spill_pending():
                start = time.monotonic()  # progress is being made: reset the grace period
                continue
            if time.monotonic() - start >= grace:
                return None

    def _fallback_write(self, oid: bytes, size: int, fill):
        """Disk-backed fallback allocation: the object's bytes in ``<spill_dir>/<oid>``,
        written through a shared writable mapping (no staging copy) and published by
        rename, where every reader (get_buffer, contains, the cross-node pull) already
        looks for file-backed objects."""
        p = self._spill_path(oid)
        tmp = p + f".fb{os.getpid()}"
        with open(tmp, "wb+") as f:
            f.truncate(max(size, 1))
            if size:
                mm = mmap.mmap(f.fileno(), size)
                try:
                    mv = memoryview(mm)
                    try:
                        fill(mv)
                    finally:
                        mv.release()
                finally:
                    mm.close()
        os.replace(tmp, p)
        self.fallback_bytes += size
        self.fallback_objects += 1

    def put_serialized(self, oid: bytes, sobj: "ser.SerializedObject", pinned: bool = True):
        off = self._alloc(oid, sobj.total, pinned)
        if off is None:
            def fill(mv):
                sobj.write_to(mv)

            self._fallback_write(oid, sobj.total, fill)
            return
        if sobj.total >= POPULATE_MIN:
            self.store.populate(off, sobj.total)
        try:
            mv = self.store.buffer(off, sobj.total)
            try:
                sobj.write_to(mv, lambda o, b: self.store.write(off + o, b))
            finally:
                mv.release()
        except BaseException:
            self.store.abort(oid)  # never leave a half-written kCreated entry behind
            raise
        self.store.seal(oid)

    def put_bytes(self, oid: bytes, data, pinned: bool = True):
        n = len(data)
        off = self._alloc(oid, n, pinned)
        if off is None:
            def fill(mv):
                mv[:n] = memoryview(data).cast("B")

            self._fallback_write(oid, n, fill)
            return
        if n >= POPULATE_MIN:
            self.store.populate(off, n)
        try:
            self.store.write(off, data)
        except BaseException:
            self.store.abort(oid)
            raise
        self.store.seal(oid)

    # ------------------------------------------------------------------ read
    def get_buffer(self, oid: bytes):
        """Pinned read-only memoryview of a sealed object, or None."""
        b = self.store.get_buffer(oid, True)
        if b is not None:
            return memoryview(b)
        p = self._spill_path(oid)
        if os.path.exists(p):
            try:
                m = _MmapBuf(p)
            except (FileNotFoundError, ValueError):
                return None
            self.restored_bytes += len(m.mv)
            return m.mv
        return None

    def contains(self, oid: bytes) -> bool:
        return self.store.contains(oid) or os.path.exists(self._spill_path(oid))

    def delete(self, oid: bytes):
        self.store.remove(oid)
        p = self._spill_path(oid)
        if self.spilled_bytes or os.path.exists(p):
            try:
                os.unlink(p)
            except FileNotFoundError:
                pass

    # ------------------------------------------------------------------ spill
    def _spill_path(self, oid: bytes) -> str:
        return os.path.join(self.spill_dir, oid.hex())

    def spill(self, oid: bytes) -> bool:
        b = self.store.get_buffer(oid, True)
        if b is None:
            return False
        try:
            mv = memoryview(b)
            p = self._spill_path(oid)
            tmp = p + f".tmp{os.getpid()}"
            with open(tmp, "wb") as f:
                f.write(mv)
            os.replace(tmp, p)
            self.spilled_bytes += len(mv)
            mv.release()
        finally:
            b.release()
        self.store.remove(oid)
        return True

    def stats(self):
        return {
            "used": self.store.used(-1),
            "capacity": self.store.capacity(-1),
            "num_objects": self.store.num_objects(),
            "evictions": self.store.evictions(),
            "spilled_bytes": self.spilled_bytes,
            "restored_bytes": self.restored_bytes,
            "fallback_bytes": self.fallback_bytes,
            "fallback_objects": self.fallback_objects,
            "waited_allocs": self.waited_allocs,
        }


def deserialize_buffer(mv, ctx=None):
    return ser.deserialize(mv, ctx)
