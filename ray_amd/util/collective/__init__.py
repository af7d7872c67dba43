"""Collective communication for ray_amd actors (RCCL over xGMI / gloo)."""

from ray_amd.util.collective.collective import (allgather, allreduce,  # noqa: F401
                                                allreduce_coalesced, alltoall, barrier,
                                                broadcast, create_collective_group,
                                                destroy_collective_group,
                                                get_collective_group_size, get_rank,
                                                init_collective_group, is_group_initialized,
                                                recv, reduce, reducescatter, send, synchronize)
from ray_amd.util.collective.collective import (allgather_multigpu,  # noqa: F401
                                                allreduce_multigpu, broadcast_multigpu,
                                                gloo_available, nccl_available,
                                                recv_multigpu, reduce_multigpu,
                                                reducescatter_multigpu, send_multigpu)
from ray_amd.util.collective.types import Backend, ReduceOp  # noqa: F401
