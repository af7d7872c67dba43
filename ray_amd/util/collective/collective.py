"""ray_amd.util.collective — collective communication between actors/tasks
(reference: python/ray/util/collective/collective.py, collective_group/nccl_collective_group.py).

Backends: "nccl" (= RCCL on ROCm, over xGMI within a node) and "gloo" (CPU). Each
named group is a torch.distributed process group created inside the member
processes; rendezvous goes through the cluster KV (rank 0 publishes a TCP
address), so groups can be declared from the driver for a set of actors
(``create_collective_group``) or joined from inside the actors
(``init_collective_group``).

MI355X note: xGMI is point-to-point (7 links/GPU) and RCCL's ring all-reduce is
per-link bound, so large tensors are cut into ``bucket_bytes`` chunks that keep
every link busy while the next chunk is being reduced (``allreduce_coalesced``).
"""

from __future__ import annotations

import os
import socket
import time
from datetime import timedelta

import torch
import torch.distributed as dist

from ray_amd.util.collective.types import Backend, ReduceOp

_groups: dict[str, "_Group"] = {}

_TORCH_OPS = {
    ReduceOp.SUM: dist.ReduceOp.SUM,
    ReduceOp.PRODUCT: dist.ReduceOp.PRODUCT,
    ReduceOp.MIN: dist.ReduceOp.MIN,
    ReduceOp.MAX: dist.ReduceOp.MAX,
}


class _Group:
    def __init__(self, name, world_size, rank, backend, pg):
        self.name = name
        self.world_size = world_size
        self.rank = rank
        self.backend = backend
        self.pg = pg


def _kv():
    from ray_amd.experimental import internal_kv

    return internal_kv


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def is_group_initialized(group_name: str = "default") -> bool:
    return group_name in _groups


def init_collective_group(world_size: int, rank: int, backend=Backend.NCCL,
                          group_name: str = "default", timeout_s: int = 600):
    """Join `group_name` from inside the current worker/actor."""
    backend = Backend(backend)
    if group_name in _groups:
        raise RuntimeError(f"collective group {group_name!r} already initialised here")
    if not (0 <= rank < world_size):
        raise ValueError("rank must be in [0, world_size)")
    kv = _kv()
    key = f"collective:{group_name}:addr"
    if rank == 0:
        from ray_amd.util import get_node_ip_address

        addr = f"{get_node_ip_address()}:{_free_port()}"
        kv._internal_kv_put(key, addr.encode(), overwrite=True, namespace="collective")
    else:
        t0 = time.time()
        while True:
            v = kv._internal_kv_get(key, namespace="collective")
            if v is not None:
                addr = v.decode()
                break
            if time.time() - t0 > timeout_s:
                raise TimeoutError(f"rendezvous for collective group {group_name} timed out")
            time.sleep(0.01)
    torch_backend = "nccl" if backend == Backend.NCCL else "gloo"
    store = dist.TCPStore(addr.split(":")[0], int(addr.split(":")[1]), world_size,
                          is_master=(rank == 0), timeout=timedelta(seconds=timeout_s))
    if torch_backend == "nccl":
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(int(os.environ.get("RAY_AMD_LOCAL_DEVICE", "0")))
    if not dist.is_initialized():
        dist.init_process_group(torch_backend, store=store, rank=rank, world_size=world_size,
                                timeout=timedelta(seconds=timeout_s))
        pg = dist.group.WORLD
    else:
        pg = dist.new_group(list(range(world_size)), backend=torch_backend)
    _groups[group_name] = _Group(group_name, world_size, rank, backend, pg)
    if rank == 0:
        # keep the store alive with the group
        _groups[group_name].store = store
    else:
        _groups[group_name].store = store


def create_collective_group(actors, world_size: int, ranks: list[int], backend=Backend.NCCL,
                            group_name: str = "default"):
    """Declare a group from the driver: every actor joins with its rank."""
    import ray_amd as ray

    if len(actors) != len(ranks) or len(actors) != world_size:
        raise ValueError("actors, ranks and world_size must agree")
    refs = []
    for a, r in zip(actors, ranks):
        refs.append(a.__ray_call__.remote(_join, world_size, r, Backend(backend).value,
                                          group_name)
                    if hasattr(a, "__ray_call__") else None)
    if any(x is None for x in refs):
        raise TypeError("actors must expose __ray_call__ (use ray_amd.remote classes)")
    ray.get(refs)


def _join(_self, world_size, rank, backend, group_name):
    init_collective_group(world_size, rank, backend, group_name)
    return True


def destroy_collective_group(group_name: str = "default"):
    g = _groups.pop(group_name, None)
    if g is None:
        return
    if g.pg is not dist.group.WORLD:
        dist.destroy_process_group(g.pg)
    elif not _groups:
        dist.destroy_process_group()
    if g.rank == 0:
        try:
            _kv()._internal_kv_del(f"collective:{group_name}:addr", namespace="collective")
        except Exception:
            pass


def _g(name):
    g = _groups.get(name)
    if g is None:
        raise RuntimeError(f"collective group {name!r} is not initialised in this process")
    return g


def get_rank(group_name: str = "default") -> int:
    return _groups[group_name].rank if group_name in _groups else -1


def get_collective_group_size(group_name: str = "default") -> int:
    return _groups[group_name].world_size if group_name in _groups else -1


def allreduce(tensor, group_name: str = "default", op=ReduceOp.SUM):
    g = _g(group_name)
    dist.all_reduce(tensor, op=_TORCH_OPS[op], group=g.pg)
    return tensor


def allreduce_coalesced(tensors, group_name: str = "default", op=ReduceOp.SUM,
                        bucket_bytes: int = 64 << 20):
    """All-reduce many tensors with a few large flat buckets (one kernel per bucket)."""
    g = _g(group_name)
    if not tensors:
        return tensors
    if g.backend == Backend.NCCL and all(t.is_cuda and t.is_contiguous() for t in tensors):
        # RCCL: one grouped launch over the tensors in place (ncclGroupStart/End under the
        # coalescing manager) - no flatten / unflatten copies through a staging buffer
        from torch.distributed.distributed_c10d import _coalescing_manager

        with _coalescing_manager(group=g.pg, device=tensors[0].device):
            for t in tensors:
                dist.all_reduce(t, op=_TORCH_OPS[op], group=g.pg)
        return tensors
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (dt, dev), ts in by_dtype.items():
        bucket, size = [], 0
        for t in ts + [None]:
            if t is not None:
                bucket.append(t)
                size += t.numel() * t.element_size()
            if bucket and (t is None or size >= bucket_bytes):
                flat = torch.cat([b.reshape(-1) for b in bucket])
                dist.all_reduce(flat, op=_TORCH_OPS[op], group=g.pg)
                o = 0
                for b in bucket:
                    b.copy_(flat[o:o + b.numel()].view_as(b))
                    o += b.numel()
                bucket, size = [], 0
    return tensors


def barrier(group_name: str = "default"):
    g = _g(group_name)
    if g.backend == Backend.NCCL:
        t = torch.zeros(1, device="cuda")
        dist.all_reduce(t, group=g.pg)
        torch.cuda.synchronize()
    else:
        dist.barrier(group=g.pg)


def reduce(tensor, dst_rank: int = 0, group_name: str = "default", op=ReduceOp.SUM):
    g = _g(group_name)
    dist.reduce(tensor, dst=dst_rank, op=_TORCH_OPS[op], group=g.pg)
    return tensor


def broadcast(tensor, src_rank: int = 0, group_name: str = "default"):
    g = _g(group_name)
    dist.broadcast(tensor, src=src_rank, group=g.pg)
    return tensor


def allgather(tensor_list, tensor, group_name: str = "default"):
    g = _g(group_name)
    if len(tensor_list) != g.world_size:
        raise RuntimeError("tensor_list must have world_size elements")
    dist.all_gather(tensor_list, tensor, group=g.pg)
    return tensor_list


def reducescatter(tensor, tensor_list, group_name: str = "default", op=ReduceOp.SUM):
    g = _g(group_name)
    if g.backend == Backend.NCCL:
        dist.reduce_scatter(tensor, list(tensor_list), op=_TORCH_OPS[op], group=g.pg)
    else:  # gloo has no reduce_scatter: all-reduce the concatenation and keep our slice
        flat = torch.cat([t.reshape(-1) for t in tensor_list])
        dist.all_reduce(flat, op=_TORCH_OPS[op], group=g.pg)
        n = tensor.numel()
        tensor.copy_(flat[g.rank * n:(g.rank + 1) * n].view_as(tensor))
    return tensor


def alltoall(output_list, input_list, group_name: str = "default"):
    g = _g(group_name)
    if g.backend == Backend.NCCL:
        dist.all_to_all(output_list, input_list, group=g.pg)
    else:  # gloo: pairwise isend / recv
        reqs = []
        for dst in range(g.world_size):
            if dst == g.rank:
                output_list[dst].copy_(input_list[dst])
            else:
                reqs.append(dist.isend(input_list[dst], dst, group=g.pg))
        for src in range(g.world_size):
            if src != g.rank:
                dist.recv(output_list[src], src, group=g.pg)
        for r in reqs:
            r.wait()
    return output_list


def send(tensor, dst_rank: int, group_name: str = "default"):
    g = _g(group_name)
    dist.send(tensor, dst_rank, group=g.pg)


def recv(tensor, src_rank: int, group_name: str = "default"):
    g = _g(group_name)
    dist.recv(tensor, src_rank, group=g.pg)
    return tensor


def synchronize(gpu_id: int = 0):
    if torch.cuda.is_available():
        torch.cuda.synchronize(gpu_id)


# ------------------------------------------------------------------ availability / multigpu
def gloo_available() -> bool:
    return dist.is_available() and dist.is_gloo_available()


def nccl_available() -> bool:
    """RCCL (torch's "nccl" backend on ROCm)."""
    return dist.is_available() and dist.is_nccl_available()


# The *_multigpu calls (reference: util/collective/collective.py) take one tensor per GPU
# of the calling process. This framework runs one process per GPU, so the list usually
# has one tensor; longer lists (several devices driven from one process) are reduced
# locally onto the first tensor's device, go through the one inter-process collective,
# and are copied back: the result is the same as the reference's flat (process x gpu)
# rank space for every reduce op.
def _local_reduce(tensors, op, into: int = 0):
    acc = tensors[into]
    for i, t in enumerate(tensors):
        if i == into:
            continue
        x = t.to(acc.device, non_blocking=True)
        if op == ReduceOp.SUM:
            acc.add_(x)
        elif op == ReduceOp.PRODUCT:
            acc.mul_(x)
        elif op == ReduceOp.MIN:
            torch.minimum(acc, x, out=acc)
        elif op == ReduceOp.MAX:
            torch.maximum(acc, x, out=acc)
        else:
            raise ValueError(f"unsupported reduce op {op}")
    return acc


def allreduce_multigpu(tensor_list, group_name: str = "default", op=ReduceOp.SUM):
    acc = _local_reduce(tensor_list, op)
    allreduce(acc, group_name, op)
    for t in tensor_list[1:]:
        t.copy_(acc)
    return tensor_list


def reduce_multigpu(tensor_list, dst_rank: int = 0, dst_tensor: int = 0,
                    group_name: str = "default", op=ReduceOp.SUM):
    acc = _local_reduce(tensor_list, op, into=dst_tensor)
    reduce(acc, dst_rank, group_name, op)
    return tensor_list


def broadcast_multigpu(tensor_list, src_rank: int = 0, src_tensor: int = 0,
                       group_name: str = "default"):
    g = _g(group_name)
    buf = tensor_list[src_tensor] if g.rank == src_rank else tensor_list[0]
    broadcast(buf, src_rank, group_name)
    for t in tensor_list:
        if t is not buf:
            t.copy_(buf)
    return tensor_list


def allgather_multigpu(output_tensor_lists, input_tensor_list, group_name: str = "default"):
    """output_tensor_lists[i] (one list per local tensor) receives all world * N inputs in
    global (process, local index) order."""
    g = _g(group_name)
    n = len(input_tensor_list)
    dev = input_tensor_list[0].device
    stacked = torch.stack([t.to(dev) for t in input_tensor_list])
    parts = [torch.empty_like(stacked) for _ in range(g.world_size)]
    dist.all_gather(parts, stacked, group=g.pg)
    for outs in output_tensor_lists:
        if len(outs) != g.world_size * n:
            raise RuntimeError("each output list needs world_size * len(input_tensor_list) "
                               "tensors")
        for p in range(g.world_size):
            for k in range(n):
                outs[p * n + k].copy_(parts[p][k])
    return output_tensor_lists


def reducescatter_multigpu(output_tensor_list, input_tensor_lists, group_name: str = "default",
                           op=ReduceOp.SUM):
    """Local tensor i receives the reduction of chunk (rank * N + i) of every input list."""
    g = _g(group_name)
    n = len(output_tensor_list)
    chunks = len(input_tensor_lists[0])
    if chunks != g.world_size * n:
        raise RuntimeError("each input list needs world_size * len(output_tensor_list) tensors")
    dev = output_tensor_list[0].device
    per = [torch.stack([t.to(dev) for t in lst]) for lst in input_tensor_lists]
    flat = _local_reduce(per, op)
    dist.all_reduce(flat, op=_TORCH_OPS[op], group=g.pg)
    for i, out in enumerate(output_tensor_list):
        out.copy_(flat[g.rank * n + i])
    return output_tensor_list


def send_multigpu(tensor, dst_rank: int, dst_gpu_index: int = 0,
                  group_name: str = "default", n_elements: int = 0):
    t = tensor.reshape(-1)[:n_elements] if n_elements else tensor
    send(t.contiguous(), dst_rank, group_name)


def recv_multigpu(tensor, src_rank: int, src_gpu_index: int = 0,
                  group_name: str = "default", n_elements: int = 0):
    if n_elements:
        buf = torch.empty(n_elements, dtype=tensor.dtype, device=tensor.device)
        recv(buf, src_rank, group_name)
        tensor.reshape(-1)[:n_elements].copy_(buf)
        return tensor
    return recv(tensor, src_rank, group_name)
