"""``ray_amd.workflow`` — durable DAG execution (parity: ``ray.workflow``)."""

from ray_amd.workflow.api import (  # noqa: F401
    EventListener,
    TimerListener,
    WorkflowCancellationError,
    WorkflowError,
    WorkflowExecutionError,
    WorkflowNotFoundError,
    WorkflowStatus,
    cancel,
    continuation,
    delete,
    get_metadata,
    get_output,
    get_output_async,
    get_status,
    init,
    list_all,
    options,
    resume,
    resume_all,
    resume_async,
    run,
    run_async,
    sleep,
    wait_for_event,
)
from ray_amd.workflow.context import get_current_task_id, get_current_workflow_id  # noqa: F401
