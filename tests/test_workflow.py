"""Workflow tests (modelled on python/ray/workflow/tests/test_basic_workflows*.py,
test_recovery.py, test_dynamic_workflow_ref.py, test_cancellation.py)."""

import os
import time

import pytest

import ray_amd as ray
from ray_amd import workflow
from ray_amd.dag import InputNode


@pytest.fixture(scope="module")
def cluster(tmp_path_factory):
    ray.init(num_cpus=4)
    workflow.init(str(tmp_path_factory.mktemp("wf")))
    yield
    ray.shutdown()


@ray.remote
def add(a, b):
    return a + b


@ray.remote
def mul(a, b):
    return a * b


def _bump(path):
    n = int(open(path).read()) if os.path.exists(path) else 0
    with open(path, "w") as f:
        f.write(str(n + 1))
    return n + 1


def test_run_and_output(cluster):
    with InputNode() as x:
        dag = mul.bind(add.bind(x, 1), add.bind(x, 2))
    assert workflow.run(dag, 3, workflow_id="wf_basic", metadata={"k": "v"}) == 20
    assert workflow.get_status("wf_basic") == workflow.WorkflowStatus.SUCCESSFUL
    assert workflow.get_output("wf_basic") == 20
    assert workflow.get_output("wf_basic", task_id="add") == 4
    assert workflow.get_output("wf_basic", task_id="add_1") == 5
    assert ("wf_basic", workflow.WorkflowStatus.SUCCESSFUL) in workflow.list_all()
    md = workflow.get_metadata("wf_basic")
    assert md["user_metadata"] == {"k": "v"} and md["stats"]["end_time"] >= md["stats"]["start_time"]
    assert workflow.get_metadata("wf_basic", "mul")["task_id"] == "mul"
    # re-running a finished workflow id returns the stored output
    assert workflow.run(dag, 3, workflow_id="wf_basic") == 20


def test_resume_skips_committed_steps(cluster, tmp_path):
    counter = str(tmp_path / "count")
    flag = str(tmp_path / "fail")
    open(flag, "w").close()

    @ray.remote
    def expensive(x):
        _bump(counter)
        return x * 10

    @ray.remote
    def flaky(x):
        if os.path.exists(flag):
            raise RuntimeError("transient")
        return x + 1

    dag = flaky.bind(expensive.options(**workflow.options(task_id="exp")).bind(4))
    with pytest.raises(Exception):
        workflow.run(dag, workflow_id="wf_resume")
    assert workflow.get_status("wf_resume") == workflow.WorkflowStatus.FAILED
    os.unlink(flag)
    assert workflow.resume("wf_resume") == 41
    assert open(counter).read() == "1"  # "exp" ran once: its checkpoint was reused
    assert workflow.get_status("wf_resume") == workflow.WorkflowStatus.SUCCESSFUL


@ray.remote
def fact(n, acc=1):
    if n <= 1:
        return acc
    return workflow.continuation(fact.bind(n - 1, acc * n))


def test_continuation_and_catch(cluster):
    assert workflow.run(fact.bind(6), workflow_id="wf_fact") == 720

    @ray.remote
    def bad():
        raise ValueError("x")

    out, err = workflow.run(bad.options(**workflow.options(catch_exceptions=True)).bind(),
                            workflow_id="wf_catch")
    assert out is None and isinstance(err, ValueError)


def test_cancel_and_delete(cluster):
    @ray.remote
    def slow():
        time.sleep(60)
        return 1

    ref = workflow.run_async(slow.bind(), workflow_id="wf_cancel")
    t0 = time.time()
    while workflow.get_status("wf_cancel") != workflow.WorkflowStatus.RUNNING:
        assert time.time() - t0 < 30
        time.sleep(0.05)
    workflow.cancel("wf_cancel")
    assert workflow.get_status("wf_cancel") == workflow.WorkflowStatus.CANCELED
    with pytest.raises(Exception):
        ray.get(ref, timeout=30)
    workflow.delete("wf_cancel")
    with pytest.raises(workflow.WorkflowNotFoundError):
        workflow.get_status("wf_cancel")


def test_sleep_and_event(cluster):
    t0 = time.time()
    workflow.run(workflow.sleep(0.3), workflow_id="wf_sleep")
    assert time.time() - t0 >= 0.3
    ev = workflow.wait_for_event(workflow.TimerListener, time.time() + 0.2)
    workflow.run(ev, workflow_id="wf_event")
    assert workflow.get_status("wf_event") == workflow.WorkflowStatus.SUCCESSFUL
