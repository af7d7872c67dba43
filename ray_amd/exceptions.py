"""Exception hierarchy (parity with python/ray/exceptions.py)."""

from __future__ import annotations

import traceback


class RayError(Exception):
    """Super class of all ray_amd exception types."""


class RaySystemError(RayError):
    def __init__(self, client_exc, traceback_str=None):
        self.client_exc = client_exc
        self.traceback_str = traceback_str
        super().__init__(str(client_exc))


class RayTaskError(RayError):
    """A task raised. ``cause`` is the original exception; ``as_instanceof_cause`` builds an
    exception that is also an instance of the cause's class (reference: exceptions.py)."""

    def __init__(self, function_name, traceback_str, cause, proctitle=None, pid=None, ip=None,
                 actor_repr=None, actor_id=None):
        self.function_name = function_name
        self.traceback_str = traceback_str
        self.cause = cause
        self.pid = pid
        self.ip = ip
        self.actor_repr = actor_repr
        self.actor_id = actor_id
        super().__init__(self._msg())

    def _msg(self):
        return (f"{type(self.cause).__name__} in {self.function_name}() "
                f"(pid={self.pid}):\n{self.traceback_str}")

    def __reduce__(self):
        return (RayTaskError, (self.function_name, self.traceback_str, self.cause, None,
                               self.pid, self.ip, self.actor_repr, self.actor_id))

    def __str__(self):
        return self._msg()

    def as_instanceof_cause(self):
        cause_cls = type(self.cause)
        if issubclass(RayTaskError, cause_cls) or isinstance(self.cause, RayTaskError):
            return self
        try:
            name = f"RayTaskError({cause_cls.__name__})"
            cls = type(name, (RayTaskError, cause_cls), {})
            err = cls.__new__(cls)
            RayTaskError.__init__(err, self.function_name, self.traceback_str, self.cause,
                                  None, self.pid, self.ip, self.actor_repr, self.actor_id)
            try:
                err.args = self.cause.args
            except Exception:
                pass
            # keep attributes of the cause reachable
            for k, v in getattr(self.cause, "__dict__", {}).items():
                if not hasattr(err, k):
                    try:
                        setattr(err, k, v)
                    except Exception:
                        pass
            return err
        except TypeError:
            return self

    @staticmethod
    def from_exception(e, function_name, pid=None, actor_repr=None):
        tb = "".join(traceback.format_exception(type(e), e, e.__traceback__))
        return RayTaskError(function_name, tb, e, pid=pid, actor_repr=actor_repr)


class RayActorError(RayError):
    def __init__(self, actor_id=None, error_msg="The actor died unexpectedly before finishing "
                 "this task.", preempted=False):
        self.actor_id = actor_id
        self.error_msg = error_msg
        self.preempted = preempted
        super().__init__(error_msg)

    def __reduce__(self):
        return (RayActorError, (self.actor_id, self.error_msg, self.preempted))


class ActorDiedError(RayActorError):
    pass


class ActorUnavailableError(RayActorError):
    pass


class ActorUnschedulableError(RayError):
    pass


class TaskUnschedulableError(RayError):
    pass


class TaskPlacementGroupRemoved(TaskUnschedulableError):
    """The placement group a task was scheduled into was removed before it ran."""


class ActorPlacementGroupRemoved(ActorUnschedulableError):
    """The placement group an actor was scheduled into was removed before it started."""


class UserCodeException(RayError):
    """An exception raised by user code run by a library (Ray Data UDFs and the like)."""


class RpcError(RayError):
    """A control-plane RPC failed (``rpc_code`` carries the transport's status, if any)."""

    def __init__(self, message, rpc_code=None):
        self.rpc_code = rpc_code
        super().__init__(message)

    def __reduce__(self):
        return (RpcError, (str(self), self.rpc_code))


class ObjectRefStreamEndOfStreamError(RayError, StopIteration):
    """Reading past the last item of a streaming generator's ObjectRef stream."""


class WorkerCrashedError(RayError):
    def __init__(self, msg="The worker died unexpectedly while executing this task."):
        super().__init__(msg)


class TaskCancelledError(RayError):
    def __init__(self, task_id=None):
        self.task_id = task_id
        super().__init__(f"Task {task_id} was cancelled")

    def __reduce__(self):
        return (TaskCancelledError, (self.task_id,))


class GetTimeoutError(RayError, TimeoutError):
    pass


class ObjectLostError(RayError):
    def __init__(self, object_ref_hex="", owner_address="", call_site=""):
        self.object_ref_hex = object_ref_hex
        super().__init__(f"Object {object_ref_hex} is lost")

    def __reduce__(self):
        return (type(self), (self.object_ref_hex,))


class OwnerDiedError(ObjectLostError):
    pass


class ObjectFreedError(ObjectLostError):
    """The object was manually freed with ``ray_amd.internal.free``."""

    def __str__(self):
        return (f"Object {self.object_ref_hex} was manually freed using the internal `free` "
                "call. Please ensure that `free` is only called once the object is no "
                "longer needed.")


class ReferenceCountingAssertionError(ObjectLostError, AssertionError):
    """An object was deleted while a reference to it still existed."""


class ObjectFetchTimedOutError(ObjectLostError):
    pass


class ReferenceCountingAssertionError(ObjectLostError):
    pass


class ObjectReconstructionFailedError(ObjectLostError):
    """The object was lost and re-executing the task that created it failed
    (reference: python/ray/exceptions.py:581)."""

    def __init__(self, object_ref_hex="", reason="", *a):
        self.reason = reason
        super().__init__(object_ref_hex)
        if reason:
            self.args = (f"Object {object_ref_hex} is lost and could not be reconstructed: "
                         f"{reason}",)

    def __str__(self):
        return self.args[0] if self.args else super().__str__()

    def __reduce__(self):
        return (type(self), (self.object_ref_hex, self.reason))


class ObjectReconstructionFailedMaxAttemptsExceededError(ObjectReconstructionFailedError):
    """Lineage re-execution would exceed the creating task's max_retries."""


class ObjectReconstructionFailedLineageEvictedError(ObjectReconstructionFailedError):
    """The creating task's spec (lineage) was evicted, so it cannot be re-executed."""


class ObjectStoreFullError(RayError):
    pass


class OutOfMemoryError(RayError):
    pass


class OutOfDiskError(RayError):
    pass


class NodeDiedError(RayError):
    pass


class LocalRayletDiedError(RayError):
    pass


class PendingCallsLimitExceeded(RayError):
    pass


class RuntimeEnvSetupError(RayError):
    pass


class CrossLanguageError(RayError):
    pass


class AsyncioActorExit(RayError):
    pass


class PlasmaObjectNotAvailable(RayError):
    pass


class RayChannelError(RayError):
    pass


class RayChannelTimeoutError(RayChannelError, TimeoutError):
    pass


class RayCgraphCapacityExceeded(RayChannelError):
    pass


class CollectiveError(RayError):
    pass
