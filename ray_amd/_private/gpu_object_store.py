"""HBM object store: GPU tensors as first-class objects, shared zero-copy between
processes on a node (north-star component; the reference has no equivalent —
Ray copies GPU tensors to host plasma on ray.put).

Layout:
  * one arena per GPU: ``hipMalloc`` by a small holder process (spawned by the
    raylet, which itself never initialises HIP), exported once with
    ``hipIpcGetMemHandle`` (dmabuf IPC on this ROCm stack);
  * the arena's allocator + object table live in the node's shared-memory store
    (``_core.ShmStore`` device heaps: same native allocator as host objects);
  * ``ray.put(cuda_tensor)`` / returning a CUDA tensor from a task: one D2D copy into
    the arena on the caller's stream, NO host block: an event is recorded after the
    copy and a per-process sealer thread seals the entry when the event completes;
    readers wait for the seal (the producer never synchronises);
  * ``ray.get`` in any process that can see that GPU: open the arena handle once, then
    wrap ``base + offset`` as a DLPack tensor (kDLROCM) — no copy, no host bounce. The
    reader pins the entry; the DLPack deleter drops the pin when the last torch view
    dies. ``RAY_AMD_HBM_COPY_ON_GET=1`` hands readers private copies instead (objects
    are immutable; torch has no read-only tensors, so zero-copy readers must not write);
  * a reader on ANOTHER GPU it cannot address (isolated HIP_VISIBLE_DEVICES) asks the
    source GPU's arena holder — which sees every GPU — for a peer copy over xGMI into
    the reader's GPU arena (an unpinned, evictable secondary copy), then maps that;
  * arena full: unpinned secondary copies are evicted (LRU); then pinned primaries are
    spilled to the host shm store (D2H) and restored by H2D on their next get.
Sub-object ids are derived from the containing object's id, so the owner frees them
(primary, secondaries, host spill copies) together with the object.
"""

from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import queue
import struct
import sys
import threading
import time

_DEFAULT_ARENA = int(os.environ.get("RAY_AMD_HBM_STORE_BYTES", str(16 << 30)))
ENABLED = os.environ.get("RAY_AMD_HBM_OBJECT_STORE", "1") == "1"
COPY_ON_GET = os.environ.get("RAY_AMD_HBM_COPY_ON_GET", "0") == "1"
# testing aid: always go through the holder's peer-copy path, even for a visible GPU
FORCE_PEER = os.environ.get("RAY_AMD_HBM_FORCE_PEER_COPY", "0") == "1"
NO_SPACE = (1 << 64) - 1
MAX_DEVICES = 16

_lock = threading.Lock()
_arenas: dict = {}  # physical device -> (base_ptr, size, local_index)
_keepalive: dict = {}
stats = {"puts": 0, "put_bytes": 0, "evicted": 0, "spilled": 0, "spilled_bytes": 0,
         "restored": 0, "peer_copies": 0, "host_fallbacks": 0}


def sub_object_id(oid: bytes, idx: int) -> bytes:
    return hashlib.blake2b(oid + struct.pack("<I", idx), digest_size=20).digest()


def secondary_id(sid: bytes, phys: int) -> bytes:
    """Id of the peer copy of sub-object `sid` in GPU `phys`'s arena."""
    return hashlib.blake2b(sid + b"sec" + struct.pack("<I", phys), digest_size=20).digest()


def spill_id(sid: bytes) -> bytes:
    """Id of the host-store copy of a spilled sub-object."""
    return hashlib.blake2b(sid + b"spill", digest_size=20).digest()


def _physical_ids():
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if vis:
        return [int(x) for x in vis.split(",") if x.strip() != ""]
    return None


def _phys_of_local(local: int) -> int:
    p = _physical_ids()
    return p[local] if p is not None and local < len(p) else local


def _local_of_phys(phys: int):
    p = _physical_ids()
    if p is None:
        return phys
    return p.index(phys) if phys in p else None


def _cw():
    from ray_amd._private import worker as W

    return W.global_worker.core


def _arena_info(phys: int) -> dict:
    return _cw().call_raylet("gpu_arena", phys, _DEFAULT_ARENA)


_session = [None]


def _check_session():
    """Arena mappings and holder connections belong to ONE ray_amd session: a new
    session (new raylet, new holders, new arenas) must not reuse stale IPC mappings.
    Called with _lock held."""
    cw = _cw()
    key = getattr(cw, "worker_id", None)
    if _session[0] == key:
        return
    from ray_amd.ops import _lib

    for base, _, _ in _arenas.values():
        try:
            _lib.lib().ra_arena_close(base)
        except Exception:  # noqa: BLE001
            pass
    _arenas.clear()
    for c in _holder_conns.values():
        try:
            c.close()
        except Exception:  # noqa: BLE001
            pass
    _holder_conns.clear()
    _session[0] = key


def _arena(phys: int):
    with _lock:
        _check_session()
        a = _arenas.get(phys)
        if a is not None:
            return a
        from ray_amd.ops import _lib

        info = _arena_info(phys)
        local = _local_of_phys(phys)
        if local is None:
            raise RuntimeError(f"GPU {phys} is not visible in this process")
        handle = bytes.fromhex(info["handle"])
        ptr = ctypes.c_void_p()
        rc = _lib.lib().ra_arena_open(local, handle, ctypes.byref(ptr))
        if rc != 0:
            raise RuntimeError(f"hipIpcOpenMemHandle failed ({rc}) for GPU {phys}")
        a = (ptr.value, info["size"], local)
        _arenas[phys] = a
        return a


# ------------------------------------------------------------------ sealing (no host block)
class _Sealer:
    """Seals arena entries once the copy that filled them has finished on the GPU.

    The producer records an event after its async copy and returns immediately; this
    thread waits on the events in order (hipEventSynchronize, GIL released by torch)
    and seals. An entry stays 'created' (invisible to get) until then."""

    def __init__(self):
        self.q: queue.Queue = queue.Queue()
        self.pending = 0
        self.cv = threading.Condition()
        self.t = threading.Thread(target=self._run, name="ray_amd-hbm-sealer", daemon=True)
        self.t.start()

    def submit(self, ev, store, sid):
        with self.cv:
            self.pending += 1
        self.q.put((ev, store, sid))

    def _run(self):
        while True:
            ev, store, sid = self.q.get()
            try:
                ev.synchronize()
                store.seal(sid)
            except Exception:  # noqa: BLE001
                try:
                    store.abort(sid)
                except Exception:  # noqa: BLE001
                    pass
            with self.cv:
                self.pending -= 1
                self.cv.notify_all()

    def flush(self, timeout=None):
        with self.cv:
            return self.cv.wait_for(lambda: self.pending == 0, timeout)


_sealer = None


def _get_sealer():
    global _sealer
    if _sealer is None:
        with _lock:
            if _sealer is None:
                _sealer = _Sealer()
    return _sealer


def flush():
    """Block until every HBM put issued by this process is sealed (tests / shutdown)."""
    if _sealer is not None:
        _sealer.flush()


# ------------------------------------------------------------------ allocation under pressure
def _copy_bytes(dst, src, n):
    from ray_amd.ops import _lib

    rc = _lib.lib().ra_copy_async(dst, src, n, None)
    if rc == 0:
        rc = _lib.lib().ra_stream_sync(None)
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed ({rc})")


def _spill_one(cw, sid: bytes, phys: int) -> bool:
    """Move a pinned primary from GPU `phys`'s arena to the host shm store (D2H)."""
    st = cw.store.store
    info = st.get(sid, True)
    if info is None:
        return False
    off, size = info[0], info[1]
    try:
        base = _arena(phys)[0]
        hid = spill_id(sid)
        if not cw.store.store.contains(hid):
            # no wait: a full host store fails this spill now (the caller tries the next
            # victim or reports the HBM store full) instead of blocking for the grace period
            hoff = cw.store._alloc(hid, size, True, wait=False)
            if hoff is None:
                st.release(sid)
                return False
            _copy_bytes(st.address() + hoff, base + off, size)  # D2H into the shm segment
            cw.store.store.seal(hid)
    except Exception:  # noqa: BLE001
        st.release(sid)
        return False
    st.release(sid)
    st.remove(sid)  # a racing reader's pin keeps the arena bytes alive until release
    stats["spilled"] += 1
    stats["spilled_bytes"] += size
    return True


def _create_on_device(cw, sid: bytes, nbytes: int, phys: int, pinned: bool = True):
    st = cw.store.store
    off = st.create(sid, nbytes, 0, phys, pinned)
    if off != NO_SPACE:
        return off
    stats["evicted"] += len(st.evict(2 * nbytes, phys))  # unpinned secondary copies
    off = st.create(sid, nbytes, 0, phys, pinned)
    if off != NO_SPACE or not pinned:
        return None if off == NO_SPACE else off
    for _ in range(4):  # spill pinned primaries to host, oldest first
        cands = st.spill_candidates(max(2 * nbytes, 256 << 20), phys)
        if not cands:
            break
        for c in cands:
            _spill_one(cw, c, phys)
        off = st.create(sid, nbytes, 0, phys, pinned)
        if off != NO_SPACE:
            return off
    return None


def reduce_cuda_tensor(t):
    """Pickle hook for CUDA tensors: copy into the HBM arena, return a descriptor."""
    if not ENABLED:
        return None
    from ray_amd._private import serialization as ser

    ctx = ser.current_context()
    cw = _cw()
    if ctx is None or ctx.object_id is None or cw is None or t.numel() == 0:
        return None
    import torch

    from ray_amd.ops import _lib

    t = t.detach()
    if not t.is_contiguous():
        t = t.contiguous()
    phys = _phys_of_local(t.device.index)
    try:
        base, size, local = _arena(phys)
    except Exception:  # noqa: BLE001
        return None
    nbytes = t.numel() * t.element_size()
    sid = sub_object_id(ctx.object_id, len(ctx.gpu))
    off = _create_on_device(cw, sid, nbytes, phys)
    if off is None:
        stats["host_fallbacks"] += 1
        return None  # arena full of pinned data even after spilling: host copy
    stream = torch.cuda.current_stream(t.device)
    rc = _lib.lib().ra_copy_async(base + off, t.data_ptr(), nbytes, stream.cuda_stream)
    if rc != 0:
        cw.store.store.abort(sid)
        return None
    ev = torch.cuda.Event()
    ev.record(stream)
    t.record_stream(stream)  # the source must outlive the async copy
    _get_sealer().submit(ev, cw.store.store, sid)
    ctx.gpu.append(sid)
    stats["puts"] += 1
    stats["put_bytes"] += nbytes
    return (_rebuild_gpu_tensor, (sid, phys, off, tuple(t.shape), str(t.dtype), nbytes))


# ------------------------------------------------------------------ DLPack (kDLROCM = 10)
class _DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int), ("device_id", ctypes.c_int)]


class _DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class _DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device", _DLDevice), ("ndim", ctypes.c_int),
                ("dtype", _DLDataType), ("shape", ctypes.POINTER(ctypes.c_int64)),
                ("strides", ctypes.POINTER(ctypes.c_int64)), ("byte_offset", ctypes.c_uint64)]


class _DLManagedTensor(ctypes.Structure):
    pass


_DELETER = ctypes.CFUNCTYPE(None, ctypes.POINTER(_DLManagedTensor))
_DLManagedTensor._fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", ctypes.c_void_p),
                             ("deleter", _DELETER)]

_DT = {"torch.float32": (2, 32), "torch.float16": (2, 16), "torch.bfloat16": (4, 16),
       "torch.float64": (2, 64), "torch.int64": (0, 64), "torch.int32": (0, 32),
       "torch.int16": (0, 16), "torch.int8": (0, 8), "torch.uint8": (1, 8), "torch.bool": (6, 8)}


def _on_delete(ptr):
    key = ctypes.addressof(ptr.contents)
    ent = _keepalive.pop(key, None)
    if ent is not None:
        store, sid = ent[0], ent[1]
        try:
            store.release(sid)
        except Exception:  # noqa: BLE001
            pass


_deleter_fn = _DELETER(_on_delete)
ctypes.pythonapi.PyCapsule_New.restype = ctypes.py_object
ctypes.pythonapi.PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]


def _wrap(store, sid, ptr, local, shape, dtype_s):
    """DLPack-wrap arena bytes whose pin the caller holds (released by the deleter)."""
    import torch

    code, bits = _DT[dtype_s]
    ndim = len(shape)
    shape_arr = (ctypes.c_int64 * max(1, ndim))(*shape)
    strides = []
    acc = 1
    for s in reversed(shape):
        strides.append(acc)
        acc *= s
    strides_arr = (ctypes.c_int64 * max(1, ndim))(*reversed(strides))
    mt = _DLManagedTensor()
    mt.dl_tensor.data = ptr
    mt.dl_tensor.device = _DLDevice(10, local)
    mt.dl_tensor.ndim = ndim
    mt.dl_tensor.dtype = _DLDataType(code, bits, 1)
    mt.dl_tensor.shape = shape_arr
    mt.dl_tensor.strides = strides_arr
    mt.dl_tensor.byte_offset = 0
    mt.manager_ctx = None
    mt.deleter = _deleter_fn
    _keepalive[ctypes.addressof(mt)] = (store, sid, mt, shape_arr, strides_arr)
    cap = ctypes.pythonapi.PyCapsule_New(ctypes.addressof(mt), b"dltensor", None)
    t = torch.utils.dlpack.from_dlpack(cap)
    if COPY_ON_GET:
        c = t.clone()
        del t  # drops the pin through the deleter
        return c
    return t


def _wait_pinned(store, sid, timeout=120.0):
    """Pin a device entry, waiting while its producer's copy is still in flight
    (state 'created'). Returns the get() tuple or None if the entry is gone."""
    deadline = time.monotonic() + timeout
    delay = 1e-5
    while True:
        info = store.get(sid, True)
        if info is not None:
            return info
        if store.state(sid) != 1:  # not created-and-pending: absent
            return None
        if time.monotonic() > deadline:
            raise TimeoutError(f"HBM object {sid.hex()} was never sealed")
        time.sleep(delay)
        delay = min(delay * 2, 1e-3)


def _restore_spilled(cw, sid, shape, dtype_s, dev_local):
    """H2D copy of a spilled sub-object into a fresh tensor on `dev_local`."""
    import torch

    hb = cw.store.get_buffer(spill_id(sid))
    if hb is None:
        return None
    import warnings

    dt = getattr(torch, dtype_s.replace("torch.", ""))
    out = torch.empty(shape, dtype=dt, device=f"cuda:{dev_local}")
    with warnings.catch_warnings():  # read-only shm view: torch only reads it here
        warnings.simplefilter("ignore")
        host = torch.frombuffer(hb, dtype=torch.uint8)
    out.view(-1).view(torch.uint8).copy_(host)
    torch.cuda.current_stream(out.device).synchronize()  # hb's pin ends with this frame
    stats["restored"] += 1
    return out


def _rebuild_gpu_tensor(sid, phys, off, shape, dtype_s, nbytes):
    import torch

    cw = _cw()
    st = cw.store.store
    local = _local_of_phys(phys)
    if local is not None and not FORCE_PEER:
        base, size, local = _arena(phys)
        info = _wait_pinned(st, sid)
        if info is not None:
            return _wrap(st, sid, base + info[0], local, shape, dtype_s)
        t = _restore_spilled(cw, sid, shape, dtype_s, local)
        if t is not None:
            return t
        from ray_amd.exceptions import ObjectLostError

        raise ObjectLostError(sid.hex())
    # the source GPU is not addressable here: peer copy into OUR GPU's arena by the
    # source arena's holder process (it sees every GPU; xGMI P2P)
    my_local = torch.cuda.current_device()
    my_phys = _phys_of_local(my_local)
    base, _, my_local = _arena(my_phys)
    sec = secondary_id(sid, my_phys)
    info = st.get(sec, True)
    if info is None:
        reply = _holder_call(phys, ("peer_copy", sid, my_phys))
        if reply[0] == "spilled":
            t = _restore_spilled(cw, sid, shape, dtype_s, my_local)
            if t is not None:
                return t
        if reply[0] != "ok":
            from ray_amd.exceptions import ObjectLostError

            raise ObjectLostError(f"{sid.hex()}: {reply}")
        stats["peer_copies"] += 1
        info = _wait_pinned(st, sec)
        if info is None:
            from ray_amd.exceptions import ObjectLostError

            raise ObjectLostError(sec.hex())
    return _wrap(st, sec, base + info[0], my_local, shape, dtype_s)


def free_sub_objects(store, oid: bytes):
    """Owner-side: drop every HBM sub-object of `oid` — primaries, peer copies on other
    GPUs and host spill copies (called when `oid` is freed)."""
    i = 0
    while True:
        sid = sub_object_id(oid, i)
        hid = spill_id(sid)
        present = store.state(sid) or store.state(hid)
        if not present:
            break
        store.remove(sid)
        store.remove(hid)
        for d in range(MAX_DEVICES):
            sec = secondary_id(sid, d)
            if store.state(sec):
                store.remove(sec)
        i += 1


# ------------------------------------------------------------------ holder RPC
_holder_conns: dict = {}


def _holder_call(phys: int, req, timeout=120.0):
    from multiprocessing.connection import Client

    info = _arena_info(phys)
    addr = info.get("sock")
    if not addr:
        raise RuntimeError(f"arena holder of GPU {phys} has no RPC socket")
    with _lock:
        _check_session()
        c = _holder_conns.get(phys)
        if c is None:
            c = _holder_conns[phys] = Client(addr, family="AF_UNIX")
        c.send(req)
        if not c.poll(timeout):
            raise TimeoutError(f"arena holder of GPU {phys} did not answer {req[0]}")
        return c.recv()


def _serve_holder(sock_path, st, phys, base, session_dir):
    """Peer-copy server of an arena holder (one thread per client connection)."""
    from multiprocessing.connection import Listener

    from ray_amd.ops import _lib

    L = _lib.lib()
    peers = {}  # dst phys -> dst base (IPC-opened)

    def dst_base(d):
        if d == phys:
            return base
        b = peers.get(d)
        if b is None:
            with open(os.path.join(session_dir, f"arena_{d}.json")) as f:
                info = json.load(f)
            ptr = ctypes.c_void_p()
            loc = _local_of_phys(d)
            rc = L.ra_arena_open(loc if loc is not None else d, bytes.fromhex(info["handle"]),
                                 ctypes.byref(ptr))
            if rc != 0:
                raise RuntimeError(f"open arena {d}: {rc}")
            b = peers[d] = ptr.value
        return b

    def handle(conn):
        while True:
            try:
                req = conn.recv()
            except (EOFError, OSError):
                return
            try:
                if req[0] == "peer_copy":
                    _, sid, d = req
                    sec = secondary_id(sid, d)
                    if st.state(sec) == 2:
                        conn.send(("ok", None))
                        continue
                    info = st.get(sid, True)
                    if info is None:
                        conn.send(("spilled",) if st.contains(spill_id(sid)) else ("lost",))
                        continue
                    try:
                        off, n = info[0], info[1]
                        doff = st.create(sec, n, 0, d, False)
                        if doff == NO_SPACE:
                            st.evict(2 * n, d)
                            doff = st.create(sec, n, 0, d, False)
                        if doff == NO_SPACE:
                            conn.send(("full",))
                            continue
                        # device-to-device across GPUs: P2P over xGMI (peer access was
                        # enabled by hipIpcMemLazyEnablePeerAccess when the arena opened)
                        rc = L.ra_copy_async(dst_base(d) + doff, base + off, n, None)
                        if rc == 0:
                            rc = L.ra_stream_sync(None)
                        if rc != 0:
                            st.abort(sec)
                            conn.send(("error", rc))
                            continue
                        st.seal(sec)
                        conn.send(("ok", doff))
                    finally:
                        st.release(sid)
                elif req[0] == "ping":
                    conn.send(("pong", phys))
                else:
                    conn.send(("error", f"unknown request {req[0]}"))
            except Exception as e:  # noqa: BLE001
                try:
                    conn.send(("error", repr(e)))
                except Exception:  # noqa: BLE001
                    return

    lis = Listener(sock_path, family="AF_UNIX")
    while True:
        c = lis.accept()
        threading.Thread(target=handle, args=(c,), daemon=True).start()


# ------------------------------------------------------------------ arena holder process
def _holder_main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, required=True)
    ap.add_argument("--size", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--store", required=True)
    ap.add_argument("--sock", default=None)
    a = ap.parse_args()
    from ray_amd._native import _core
    from ray_amd.ops import _lib

    L = _lib.lib()
    n = L.ra_ipc_handle_size()
    handle = ctypes.create_string_buffer(n)
    ptr = ctypes.c_void_p()
    local = _local_of_phys(a.device)
    rc = L.ra_arena_alloc(local if local is not None else a.device, a.size, ctypes.byref(ptr),
                          handle)
    if rc != 0:
        print(f"[ray_amd] HBM arena alloc failed on GPU {a.device}: {rc}", file=sys.stderr)
        sys.exit(1)
    st = _core.ShmStore(a.store, 0, False, 0)
    st.init_device_heap(a.device, a.size)
    info = {"device": a.device, "size": a.size, "handle": handle.raw.hex()}
    if a.sock:
        info["sock"] = a.sock
        threading.Thread(target=_serve_holder, daemon=True,
                         args=(a.sock, st, a.device, ptr.value,
                               os.path.dirname(a.out))).start()
        t0 = time.time()
        while not os.path.exists(a.sock) and time.time() - t0 < 30:
            time.sleep(0.01)
    tmp = a.out + ".tmp"
    with open(tmp, "w") as f:
        json.dump(info, f)
    os.replace(tmp, a.out)
    while True:
        time.sleep(3600)


if __name__ == "__main__":
    _holder_main()
