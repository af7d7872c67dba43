"""``ray.util.state.custom_types`` (reference: python/ray/util/state/custom_types.py): the
state strings the State API reports."""

from typing import Literal

TypeActorStatus = Literal["DEPENDENCIES_UNREADY", "PENDING_CREATION", "ALIVE", "RESTARTING",
                          "DEAD"]
ACTOR_STATUS = list(TypeActorStatus.__args__)
TypeTaskStatus = Literal["NIL", "PENDING_ARGS_AVAIL", "PENDING_NODE_ASSIGNMENT",
                         "PENDING_OBJ_STORE_MEM_AVAIL", "PENDING_ARGS_FETCH",
                         "SUBMITTED_TO_WORKER", "RUNNING", "RUNNING_IN_RAY_GET",
                         "RUNNING_IN_RAY_WAIT", "FINISHED", "FAILED"]
TASK_STATUS = list(TypeTaskStatus.__args__)
TypeNodeStatus = Literal["ALIVE", "DEAD"]
NODE_STATUS = list(TypeNodeStatus.__args__)
TypePlacementGroupStatus = Literal["PENDING", "CREATED", "REMOVED", "RESCHEDULING"]
PLACEMENT_GROUP_STATUS = list(TypePlacementGroupStatus.__args__)
TypeWorkerType = Literal["WORKER", "DRIVER", "SPILL_WORKER", "RESTORE_WORKER"]
WORKER_TYPE = list(TypeWorkerType.__args__)
TypeWorkerExitType = Literal["SYSTEM_ERROR", "INTENDED_SYSTEM_EXIT", "USER_ERROR",
                             "INTENDED_USER_EXIT", "NODE_OUT_OF_MEMORY"]
TypeTaskType = Literal["NORMAL_TASK", "ACTOR_CREATION_TASK", "ACTOR_TASK", "DRIVER_TASK"]
TASK_TYPE = list(TypeTaskType.__args__)
TypeReferenceType = Literal["ACTOR_HANDLE", "PINNED_IN_MEMORY", "LOCAL_REFERENCE",
                            "USED_BY_PENDING_TASK", "CAPTURED_IN_OBJECT", "UNKNOWN_STATUS"]
TypeJobStatus = Literal["PENDING", "RUNNING", "STOPPED", "SUCCEEDED", "FAILED"]
