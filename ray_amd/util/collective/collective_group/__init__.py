"""Group objects of ``ray.util.collective`` (reference: python/ray/util/collective/
collective_group/): ``NCCLGroup`` (RCCL on ROCm) and ``GLOOGroup`` over the named
torch.distributed groups of ``collective.py``."""

from ray_amd.util.collective.collective_group.base_collective_group import BaseGroup  # noqa
from ray_amd.util.collective.collective_group.gloo_collective_group import GLOOGroup  # noqa
from ray_amd.util.collective.collective_group.nccl_collective_group import NCCLGroup  # noqa
