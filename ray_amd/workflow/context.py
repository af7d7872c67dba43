"""The running workflow step's identity (reference: python/ray/workflow/workflow_context.py):
set by the step wrapper around the user function, read by event listeners and user code."""

from __future__ import annotations

import threading

_local = threading.local()


def _set(workflow_id, task_id):
    _local.wid, _local.task_id = workflow_id, task_id


def get_current_workflow_id():
    return getattr(_local, "wid", None)


def get_current_task_id():
    return getattr(_local, "task_id", None)
