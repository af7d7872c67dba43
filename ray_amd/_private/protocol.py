"""Wire protocol between ray_amd processes.

Frames are length-prefixed by the native IOLoop; the payload is a pickled tuple
whose first element is the message type. Two hot-path messages (TASK /
TASK_REPLY) have their own types; everything else is a generic RPC
``(REQ, rid, method, args)`` answered by ``(RESP, rid, ok, value)`` — rid 0 means
one-way. The raylet pushes notifications as ``(PUSH, topic, data)``.
(Reference: src/ray/protobuf/core_worker.proto, node_manager.proto, gcs_service.proto.)
"""

import pickle

REQ = 1
RESP = 2
PUSH = 3
HELLO = 10
TASK = 11
TASK_REPLY = 12
STREAM_ITEM = 13
# owner -> executing worker: (STREAM_ACK, tid, items consumed) for generator backpressure
STREAM_ACK = 14
STEAL = 15  # owner -> worker: give back a pipelined task that has not started yet

# task types
NORMAL_TASK = 0
ACTOR_CREATION_TASK = 1
ACTOR_TASK = 2

# return payload kinds
RET_INLINE = 0
RET_STORE = 1

# actor states (reference: gcs.proto ActorTableData.ActorState)
DEPENDENCIES_UNREADY = "DEPENDENCIES_UNREADY"
PENDING_CREATION = "PENDING_CREATION"
ALIVE = "ALIVE"
RESTARTING = "RESTARTING"
DEAD = "DEAD"


def dumps(msg) -> bytes:
    return pickle.dumps(msg, protocol=5)


loads = pickle.loads
