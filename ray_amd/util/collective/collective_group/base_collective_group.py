"""``BaseGroup`` (reference: collective_group/base_collective_group.py): one member's view
of a named collective group. Creating the object joins the group (``init_collective_group``);
the methods are the module-level collectives bound to the group's name."""

from __future__ import annotations

from ray_amd.util.collective import collective as _c
from ray_amd.util.collective.types import Backend, ReduceOp


class BaseGroup:
    _backend: Backend = None

    def __init__(self, world_size: int, rank: int, group_name: str, _join: bool = True):
        self._world_size = int(world_size)
        self._rank = int(rank)
        self._group_name = group_name
        if _join and not _c.is_group_initialized(group_name):
            _c.init_collective_group(world_size, rank, self._backend, group_name)

    @property
    def rank(self) -> int:
        return self._rank

    @property
    def world_size(self) -> int:
        return self._world_size

    @property
    def group_name(self) -> str:
        return self._group_name

    @classmethod
    def backend(cls) -> Backend:
        return cls._backend

    def destroy_group(self):
        _c.destroy_collective_group(self._group_name)

    # collectives (tensor lists are the reference's form: one tensor per call here)
    def allreduce(self, tensors, allreduce_options=None):
        op = getattr(allreduce_options, "reduceOp", ReduceOp.SUM)
        for t in _as_list(tensors):
            _c.allreduce(t, self._group_name, op)

    def barrier(self, barrier_options=None):
        _c.barrier(self._group_name)

    def reduce(self, tensors, reduce_options=None):
        op = getattr(reduce_options, "reduceOp", ReduceOp.SUM)
        root = getattr(reduce_options, "root_rank", 0)
        for t in _as_list(tensors):
            _c.reduce(t, root, self._group_name, op)

    def broadcast(self, tensors, broadcast_options=None):
        root = getattr(broadcast_options, "root_rank", 0)
        for t in _as_list(tensors):
            _c.broadcast(t, root, self._group_name)

    def allgather(self, tensor_lists, tensors, allgather_options=None):
        lists = tensor_lists if tensor_lists and isinstance(tensor_lists[0], list) \
            else [tensor_lists]
        for out, t in zip(lists, _as_list(tensors)):
            _c.allgather(out, t, self._group_name)

    def reducescatter(self, tensors, tensor_lists, reducescatter_options=None):
        op = getattr(reducescatter_options, "reduceOp", ReduceOp.SUM)
        lists = tensor_lists if tensor_lists and isinstance(tensor_lists[0], list) \
            else [tensor_lists]
        for t, inp in zip(_as_list(tensors), lists):
            _c.reducescatter(t, inp, self._group_name, op)

    def send(self, tensors, send_options=None):
        dst = getattr(send_options, "dst_rank", 0)
        for t in _as_list(tensors):
            _c.send(t, dst, self._group_name)

    def recv(self, tensors, recv_options=None):
        src = getattr(recv_options, "src_rank", 0)
        for t in _as_list(tensors):
            _c.recv(t, src, self._group_name)


def _as_list(x):
    return list(x) if isinstance(x, (list, tuple)) else [x]
