"""``GLOOGroup`` (reference: collective_group/gloo_collective_group.py): a CPU group on
the gloo backend."""

from ray_amd.util.collective.collective_group.base_collective_group import BaseGroup
from ray_amd.util.collective.types import Backend


class GLOOGroup(BaseGroup):
    _backend = Backend.GLOO
