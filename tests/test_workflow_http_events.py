"""Workflow HTTP events (reference: python/ray/workflow/tests/test_http_events*.py): a
workflow waits on HTTPListener; an external POST to the HTTPEventProvider Serve app is
answered 200 only once the event is checkpointed, unknown keys get 404, and the step's
context (workflow id, task id) is visible to listeners."""
import socket
import time

import pytest
import requests

import ray_amd as ray
from ray_amd import serve, workflow
from ray_amd.workflow.http_event_provider import HTTPListener


@pytest.fixture(scope="module")
def cluster(tmp_path_factory):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ray.init(num_cpus=6)
    serve.start(http_options={"port": port})
    workflow.init(storage=str(tmp_path_factory.mktemp("wf")))
    yield port
    serve.shutdown()
    ray.shutdown()


@ray.remote
def handle_event(ev):
    return f"got {ev[1]} for {ev[0]}"


def test_http_event_delivered_after_checkpoint(cluster):
    port = cluster
    dag = handle_event.bind(workflow.wait_for_event(HTTPListener, event_key="approve"))
    ref = workflow.run_async(dag, workflow_id="wf_http")
    url = f"http://127.0.0.1:{port}/event/send_event/wf_http"
    deadline = time.time() + 60
    status = None
    while time.time() < deadline:  # 404 until the step has registered its key
        try:
            r = requests.post(url, json={"event_key": "approve", "event_payload": "yes"},
                              timeout=30)
            status = r.status_code
        except requests.RequestException:
            status = None
        if status == 200:
            break
        time.sleep(0.2)
    assert status == 200
    assert ray.get(ref) == "got yes for approve"
    assert workflow.get_status("wf_http") == workflow.WorkflowStatus.SUCCESSFUL
    r = requests.post(url, json={"event_key": "approve", "event_payload": "again"}, timeout=30)
    assert r.status_code == 404  # nobody waits for it any more
    r = requests.post(url, json={"event_key": "x"}, timeout=30)
    assert r.status_code == 404


def test_step_context_visible(cluster):
    @ray.remote
    def whoami():
        from ray_amd.workflow.api import get_current_task_id, get_current_workflow_id

        return get_current_workflow_id(), get_current_task_id()

    assert workflow.run(whoami.bind(), workflow_id="wf_ctx") == ("wf_ctx", "whoami")
