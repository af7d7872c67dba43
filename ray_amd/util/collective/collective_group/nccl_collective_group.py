"""``NCCLGroup`` (reference: collective_group/nccl_collective_group.py): a group on the
"nccl" torch.distributed backend, which is RCCL on ROCm (xGMI inside a node)."""

from ray_amd.util.collective.collective_group.base_collective_group import BaseGroup
from ray_amd.util.collective.types import Backend


class NCCLGroup(BaseGroup):
    _backend = Backend.NCCL
