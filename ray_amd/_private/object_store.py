"""Node-local object store client (reference: plasma client + external_storage.py spilling).

Wraps the native ``_core.ShmStore``: every process on the node maps the same
/dev/shm segment, so put/get are in-process operations (no store IPC).
When the heap is full: evict unpinned secondary copies (LRU), then spill pinned
primary copies. Spilling runs OFF the put path (reference: src/ray/raylet/
local_object_manager.cc:153-176 SpillObjectUptoMaxThroughput on IO workers,
python/ray/_private/external_storage.py:246-293 fused spill files): a blocked put posts
the bytes it needs into the segment header (``spill_request``) and waits in the create
queue; the node's ``SpillManager`` thread (raylet / node agent) — also triggered by a
high-water mark — writes the LRU primaries back to back into ONE fused file
``<spill_dir>/fused-<pid>-<n>.bin`` (page-aligned offsets, write + rename), publishes each
object's location as a small pinned stub object in the store, THEN drops the object, so
a reader that misses the store always finds the stub. Spilled objects are read back
through an mmap of their fused-file range — still zero-copy. A fused file is deleted
once every object in it was freed. Without a live spill thread (a store opened
standalone) the put spills synchronously through the same fused writer.
"""

from __future__ import annotations

import hashlib
import itertools
import mmap
import os
import struct
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
    """Keeps a spill-file mapping alive while views of it exist (``off``/``size``: a range
    of a fused file; ``off`` is page-aligned)."""

    __slots__ = ("mm", "mv")

    def __init__(self, path, off=0, size=None):
        with open(path, "rb") as f:
            if size is None:
                self.mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
            elif size == 0:
                self.mm = b""
            else:
                self.mm = mmap.mmap(f.fileno(), size, access=mmap.ACCESS_READ, offset=off)
        self.mv = memoryview(self.mm)


_STUB_PREFIX = b"\xffSPL"
_STUB_FMT = struct.Struct("<QQ")  # offset, size; then the fused file's name (utf-8)
_ALIGN = mmap.ALLOCATIONGRANULARITY


def stub_id(oid: bytes) -> bytes:
    """Id of the pinned stub that records where a spilled object lives."""
    return _STUB_PREFIX + hashlib.blake2b(oid, digest_size=16).digest()


def is_stub(oid: bytes) -> bool:
    return oid[:4] == _STUB_PREFIX


def spilled_location(store, spill_dir: str, oid: bytes):
    """(path, offset, size) of a spilled object from its stub, or None."""
    b = store.get_buffer(stub_id(oid), True)
    if b is None:
        return None
    try:
        raw = bytes(memoryview(b))
    finally:
        b.release()
    off, size = _STUB_FMT.unpack_from(raw)
    return os.path.join(spill_dir, raw[_STUB_FMT.size:].decode()), off, size


def spill_fused(store, spill_dir: str, oids, max_file_bytes: int = 256 << 20) -> list:
    """Write the sealed objects ``oids`` back to back (page-aligned) into fused files of
    at most ``max_file_bytes``, publish a stub per object, then drop the objects from the
    store. Returns [(file name, [oids], bytes)] of the files written. Objects that vanished or are
    pinned by a reader mid-way are skipped."""
    files = []
    oids = [o for o in oids if not is_stub(o)]
    i = 0
    while i < len(oids):
        name = f"fused-{os.getpid()}-{next(_FUSED_SEQ)}.bin"
        path = os.path.join(spill_dir, name)
        tmp = path + ".tmp"
        placed, pos = [], 0
        store.spill_inflight_add(1)
        try:
            with open(tmp, "wb") as f:
                while i < len(oids) and (not placed or pos < max_file_bytes):
                    oid = oids[i]
                    i += 1
                    b = store.get_buffer(oid, True)
                    if b is None:
                        continue
                    try:
                        mv = memoryview(b)
                        n = len(mv)
                        if pos % _ALIGN:
                            pad = _ALIGN - pos % _ALIGN
                            f.write(b"\0" * pad)
                            pos += pad
                        f.write(mv)
                        mv.release()
                    finally:
                        b.release()
                    placed.append((oid, pos, n))
                    pos += n
            os.replace(tmp, path)
            with open(path + ".idx", "w") as f:  # manifest for the node's GC pass
                f.write("\n".join(o.hex() for o, _, _ in placed))
            done, nbytes = [], 0
            for oid, off, n in placed:
                sid = stub_id(oid)
                rec = _STUB_FMT.pack(off, n) + name.encode()
                try:
                    so = store.create(sid, len(rec), 0, -1, True)
                except RuntimeError:  # spilled concurrently by another process
                    continue
                if so == NO_SPACE:  # no room even for the stub: keep the object in memory
                    continue
                store.write(so, rec)
                store.seal(sid)
                store.remove(oid)
                done.append(oid)
                nbytes += n
            store.spilled_total_add(nbytes)
            files.append((name, done, nbytes))
        finally:
            store.spill_inflight_add(-1)
    return files


_FUSED_SEQ = itertools.count()


class SpillManager:
    """The node's spill thread (raylet / node agent): serves blocked puts' requests and a
    high-water mark (RAY_AMD_SPILL_HIGH_WATER, fraction of the host heap, default 0.9)
    by fusing LRU pinned primaries into spill files; deletes a fused file once all its
    objects were freed."""

    def __init__(self, store, spill_dir: str, high_water: float | None = None,
                 fuse_bytes: int | None = None):
        self.store, self.spill_dir = store, spill_dir
        self.high_water = float(os.environ.get("RAY_AMD_SPILL_HIGH_WATER", "0.9")) \
            if high_water is None else high_water
        self.fuse_bytes = int(fuse_bytes or os.environ.get("RAY_AMD_SPILL_FUSE_BYTES",
                                                           256 << 20))
        self.min_spill = int(os.environ.get("RAY_AMD_MIN_SPILLING_SIZE", 100 << 20))
        self.stop_ev = threading.Event()
        self.spilled_objects = 0
        self.t = threading.Thread(target=self._run, name="spill-manager", daemon=True)

    def start(self):
        self.store.set_spiller(os.getpid())
        self.t.start()
        return self

    def stop(self):
        self.stop_ev.set()
        self.t.join(timeout=5)

    def _run(self):
        import time

        last_gc = time.monotonic()
        while not self.stop_ev.is_set():
            self.store.spiller_beat()
            want = self.store.spill_take()
            cap = self.store.capacity(-1)
            over = self.store.used(-1) - int(self.high_water * cap)
            target = 0
            if want or over > 0:
                # spill at least min_spill bytes per round, down to 10 % below the high
                # water mark: fewer, larger fused files (reference: min_spilling_size)
                target = max(2 * want, over + cap // 10, self.min_spill)
            if target > 0:
                try:
                    cands = [c for c in self.store.spill_candidates(target, -1)
                             if not is_stub(c)]
                    for _name, oids, _n in spill_fused(self.store, self.spill_dir, cands,
                                                       self.fuse_bytes):
                        self.spilled_objects += len(oids)
                except Exception:  # noqa: BLE001 - keep serving; the put path falls back
                    pass
                continue
            if time.monotonic() - last_gc > 1.0:
                self.gc()
                last_gc = time.monotonic()
            self.stop_ev.wait(0.005)

    def gc(self):
        """Delete every fused file (written by any process of the node) none of whose
        objects is still spilled: their stubs are gone."""
        gc_fused_files(self.store, self.spill_dir)


def gc_fused_files(store, spill_dir: str) -> int:
    removed = 0
    try:
        names = [n for n in os.listdir(spill_dir) if n.endswith(".bin.idx")]
    except FileNotFoundError:
        return 0
    for idx in names:
        p = os.path.join(spill_dir, idx)
        try:
            with open(p) as f:
                oids = [bytes.fromhex(x) for x in f.read().split()]
        except (OSError, ValueError):
            continue
        if any(store.contains(stub_id(o)) for o in oids):
            continue
        for q in (p[:-len(".idx")], p):
            try:
                os.unlink(q)
            except OSError:
                pass
        removed += 1
    return removed


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
    def _try_make_room(self, oid: bytes, size: int, pinned: bool, device: int,
                       request: bool = True) -> int:
        off = self.store.create(oid, size, 0, device, pinned)
        if off != NO_SPACE:
            return off
        # 1) evict unpinned LRU copies
        self.store.evict(size * 2, device)
        off = self.store.create(oid, size, 0, device, pinned)
        if off != NO_SPACE or device >= 0:
            return off
        # 2) spill pinned primary copies: asked of the node's spill thread (the caller
        # waits in the create queue), or done here when no spill thread is alive
        if self.store.live_spiller(2000):
            # first attempt, or a retry after the previous spill finished without making
            # room: (re)post the request; otherwise the spill in flight is awaited
            if request or self.store.spill_inflight() == 0:
                self.store.spill_request(size)
            return NO_SPACE
        for _ in range(8):
            cands = [c for c in self.store.spill_candidates(max(size * 2, 64 << 20), device)
                     if not is_stub(c)]
            if not cands:
                break
            for _name, _oids, n in spill_fused(self.store, self.spill_dir, cands):
                self.spilled_bytes += n
            off = self.store.create(oid, size, 0, device, pinned)
            if off != NO_SPACE:
                return off
        return NO_SPACE

    def _spill_pending(self) -> bool:
        """A spill that will free space is requested or in progress on this node (the
        shared segment's counters: no directory scan)."""
        return self.store.spill_inflight() > 0

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
            off = self._try_make_room(oid, size, pinned, device, request=False)
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
        loc = spilled_location(self.store, self.spill_dir, oid)
        if loc is not None:
            try:
                m = _MmapBuf(*loc)
            except (FileNotFoundError, ValueError, OSError):
                return None
            self.restored_bytes += len(m.mv)
            return m.mv
        p = self._spill_path(oid)  # disk-backed fallback allocation (_fallback_write)
        if os.path.exists(p):
            try:
                m = _MmapBuf(p)
            except (FileNotFoundError, ValueError):
                return None
            self.restored_bytes += len(m.mv)
            return m.mv
        return None

    def contains(self, oid: bytes) -> bool:
        return self.store.contains(oid) or self.store.contains(stub_id(oid)) or \
            os.path.exists(self._spill_path(oid))

    def delete(self, oid: bytes):
        self.store.remove(oid)
        self.store.remove(stub_id(oid))  # its fused file goes when all its objects went
        p = self._spill_path(oid)
        if os.path.exists(p):
            try:
                os.unlink(p)
            except FileNotFoundError:
                pass

    # ------------------------------------------------------------------ spill
    def _spill_path(self, oid: bytes) -> str:
        return os.path.join(self.spill_dir, oid.hex())

    def spill(self, oid: bytes) -> bool:
        """Spill one object now (a fused file of one)."""
        files = spill_fused(self.store, self.spill_dir, [oid])
        ok = bool(files and files[0][1])
        if ok:
            self.spilled_bytes += files[0][2]
        return ok

    def stats(self):
        return {
            "used": self.store.used(-1),
            "capacity": self.store.capacity(-1),
            "num_objects": self.store.num_objects(),
            "evictions": self.store.evictions(),
            # node-wide (the spill thread's and every process's spills: segment counter)
            "spilled_bytes": max(self.spilled_bytes, self.store.spilled_total_add(0)),
            "restored_bytes": self.restored_bytes,
            "fallback_bytes": self.fallback_bytes,
            "fallback_objects": self.fallback_objects,
            "waited_allocs": self.waited_allocs,
        }


def deserialize_buffer(mv, ctx=None):
    return ser.deserialize(mv, ctx)
