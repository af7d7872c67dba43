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
