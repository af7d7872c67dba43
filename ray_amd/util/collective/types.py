"""Collective types (reference: python/ray/util/collective/types.py)."""

from enum import Enum


class Backend(str, Enum):
    NCCL = "nccl"  # RCCL on ROCm
    GLOO = "gloo"
    RCCL = "nccl"

    @classmethod
    def _missing_(cls, value):
        if isinstance(value, str):
            v = value.lower()
            if v in ("nccl", "rccl"):
                return cls.NCCL
            if v == "gloo":
                return cls.GLOO
        return None


class ReduceOp(Enum):
    SUM = 0
    PRODUCT = 1
    MIN = 2
    MAX = 3


# per-call options of the group objects (collective_group/base_collective_group.py)
from dataclasses import dataclass  # noqa: E402

unset_timeout_ms = 30 * 60 * 1000


@dataclass
class AllReduceOptions:
    reduceOp: ReduceOp = ReduceOp.SUM
    timeout_ms: int = unset_timeout_ms


@dataclass
class BarrierOptions:
    timeout_ms: int = unset_timeout_ms


@dataclass
class ReduceOptions:
    reduceOp: ReduceOp = ReduceOp.SUM
    root_rank: int = 0
    root_tensor: int = 0
    timeout_ms: int = unset_timeout_ms


@dataclass
class AllGatherOptions:
    timeout_ms: int = unset_timeout_ms


@dataclass
class BroadcastOptions:
    root_rank: int = 0
    root_tensor: int = 0
    timeout_ms: int = unset_timeout_ms


@dataclass
class ReduceScatterOptions:
    reduceOp: ReduceOp = ReduceOp.SUM
    timeout_ms: int = unset_timeout_ms


@dataclass
class SendOptions:
    dst_rank: int = 0
    dst_gpu_index: int = 0
    n_elements: int = 0
    timeout_ms: int = unset_timeout_ms


@dataclass
class RecvOptions:
    src_rank: int = 0
    src_gpu_index: int = 0
    n_elements: int = 0
    unset_timeout_ms: int = unset_timeout_ms
