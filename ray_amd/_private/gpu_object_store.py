"""HBM object store: GPU tensors as first-class objects, shared zero-copy between
processes on a node (north-star component; the reference has no equivalent —
Ray copies GPU tensors to host plasma on ray.put).

Layout:
  * one arena per GPU: ``hipMalloc`` by a small holder process (spawned by the
    raylet, which itself never initialises HIP), exported once with
    ``hipIpcGetMemHandle`` (dmabuf IPC on this ROCm stack);
  * the arena's allocator + object table live in the node's shared-memory store
    (``_core.ShmStore`` device heaps: same native allocator as host objects);
  * ``ray.put(cuda_tensor)`` / returning a CUDA tensor from a task: one D2D
    copy into the arena (HBM→HBM at ~TB/s), descriptor pickled in-band;
  * ``ray.get`` in any process that can see that GPU: open the arena handle
    once, then wrap ``base + offset`` as a DLPack tensor (kDLROCM) — no copy,
    no host bounce. The reader pins the entry; the pin is dropped by the
    DLPack deleter when the last torch view dies.
Sub-object ids are derived from the containing object's id, so the owner frees
them together with the object.
"""

from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import struct
import sys
import threading
import time

_DEFAULT_ARENA = int(os.environ.get("RAY_AMD_HBM_STORE_BYTES", str(16 << 30)))
ENABLED = os.environ.get("RAY_AMD_HBM_OBJECT_STORE", "1") == "1"

_lock = threading.Lock()
_arenas: dict = {}  # physical device -> (base_ptr, size, local_index)
_keepalive: dict = {}


def sub_object_id(oid: bytes, idx: int) -> bytes:
    return hashlib.blake2b(oid + struct.pack("<I", idx), digest_size=20).digest()


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


def _arena(phys: int):
    with _lock:
        a = _arenas.get(phys)
        if a is not None:
            return a
        from ray_amd._private import worker as W
        from ray_amd.ops import _lib

        cw = W.global_worker.core
        info = cw.call_raylet("gpu_arena", phys, _DEFAULT_ARENA)
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


def reduce_cuda_tensor(t):
    """Pickle hook for CUDA tensors: copy into the HBM arena, return a descriptor."""
    if not ENABLED:
        return None
    from ray_amd._private import serialization as ser
    from ray_amd._private import worker as W

    ctx = ser.current_context()
    cw = W.global_worker.core
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
    except Exception:
        return None
    nbytes = t.numel() * t.element_size()
    sid = sub_object_id(ctx.object_id, len(ctx.gpu))
    off = cw.store.store.create(sid, nbytes, 0, phys, True)
    if off == (1 << 64) - 1:
        return None  # arena full: caller falls back to a host copy
    stream = torch.cuda.current_stream(t.device)
    rc = _lib.lib().ra_copy_async(base + off, t.data_ptr(), nbytes, stream.cuda_stream)
    if rc != 0:
        cw.store.store.remove(sid)
        return None
    stream.synchronize()
    cw.store.store.seal(sid)
    ctx.gpu.append(sid)
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
        except Exception:
            pass


_deleter_fn = _DELETER(_on_delete)
ctypes.pythonapi.PyCapsule_New.restype = ctypes.py_object
ctypes.pythonapi.PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]


def _rebuild_gpu_tensor(sid, phys, off, shape, dtype_s, nbytes):
    import torch

    from ray_amd._private import worker as W

    cw = W.global_worker.core
    base, size, local = _arena(phys)
    info = cw.store.store.get(sid, True)  # pin
    if info is None:
        from ray_amd.exceptions import ObjectLostError

        raise ObjectLostError(sid.hex())
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
    mt.dl_tensor.data = base + off
    mt.dl_tensor.device = _DLDevice(10, local)
    mt.dl_tensor.ndim = ndim
    mt.dl_tensor.dtype = _DLDataType(code, bits, 1)
    mt.dl_tensor.shape = shape_arr
    mt.dl_tensor.strides = strides_arr
    mt.dl_tensor.byte_offset = 0
    mt.manager_ctx = None
    mt.deleter = _deleter_fn
    _keepalive[ctypes.addressof(mt)] = (cw.store.store, sid, mt, shape_arr, strides_arr)
    cap = ctypes.pythonapi.PyCapsule_New(ctypes.addressof(mt), b"dltensor", None)
    t = torch.utils.dlpack.from_dlpack(cap)
    return t


def free_sub_objects(store, oid: bytes):
    """Owner-side: drop every HBM sub-object of `oid` (called when `oid` is freed)."""
    i = 0
    while True:
        sid = sub_object_id(oid, i)
        if not store.state(sid):
            break
        store.remove(sid)
        i += 1


# ------------------------------------------------------------------ arena holder process
def _holder_main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, required=True)
    ap.add_argument("--size", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--store", required=True)
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
    tmp = a.out + ".tmp"
    with open(tmp, "w") as f:
        json.dump({"device": a.device, "size": a.size, "handle": handle.raw.hex()}, f)
    os.replace(tmp, a.out)
    while True:
        time.sleep(3600)


if __name__ == "__main__":
    _holder_main()
