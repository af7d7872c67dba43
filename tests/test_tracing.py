"""Distributed tracing (reference: python/ray/tests/test_tracing.py with the
setup_local_tmp_tracing hook): submit and execute spans for tasks, nested tasks and actor
calls, linked into one trace across processes, plus user spans."""
import os

import pytest

import ray_amd as ray
from ray_amd.util import tracing


@pytest.fixture
def traced(tmp_path, monkeypatch):
    d = str(tmp_path / "spans")
    monkeypatch.setenv("RAY_AMD_TRACING_DIR", d)
    if ray.is_initialized():
        ray.shutdown()
    ray.init(num_cpus=2, _tracing_startup_hook=(
        "ray_amd.util.tracing.setup_local_tmp_tracing:setup_tracing"))
    yield d
    ray.shutdown()
    tracing.disable()


def test_task_and_actor_spans_form_one_trace(traced):
    @ray.remote
    def leaf(x):
        with tracing.span("inner-work", step=1):
            return x + 1

    @ray.remote
    def parent(x):
        return ray.get(leaf.remote(x)) * 2

    @ray.remote
    class A:
        def f(self):
            return os.getpid()

        def boom(self):
            raise ValueError("no")

    assert ray.get(parent.remote(1)) == 4
    a = A.remote()
    ray.get(a.f.remote())
    with pytest.raises(ValueError):
        ray.get(a.boom.remote())
    ray.shutdown()  # flush
    spans = tracing.read_spans(traced)
    by_name = {}
    for s in spans:  # task names are qualified (test_fn.<locals>.parent): key by the tail
        head, _, tail = s["name"].partition(" ")
        by_name.setdefault(head.split(".")[-1] + (" " + tail if tail else ""), []).append(s)
    p_sub = by_name["parent ray.remote"][0]
    p_exe = by_name["parent ray.remote_worker"][0]
    l_sub = by_name["leaf ray.remote"][0]
    l_exe = by_name["leaf ray.remote_worker"][0]
    inner = by_name["inner-work"][0]
    # one trace; each execution is the child of its submission; nesting across processes
    tid = p_sub["context"]["trace_id"]
    assert all(s["context"]["trace_id"] == tid for s in (p_exe, l_sub, l_exe, inner))
    assert p_exe["parent_id"] == p_sub["context"]["span_id"]
    assert l_sub["parent_id"] == p_exe["context"]["span_id"]
    assert l_exe["parent_id"] == l_sub["context"]["span_id"]
    assert inner["parent_id"] == l_exe["context"]["span_id"]
    assert inner["attributes"]["step"] == 1
    assert p_exe["attributes"]["ray.pid"] != p_sub["attributes"]["ray.pid"]
    assert p_exe["start_time"] <= p_exe["end_time"]
    assert by_name["f ray.remote_worker"][0]["attributes"]["ray.actor_id"]
    assert by_name["boom ray.remote_worker"][0]["status"]["status_code"] == "ERROR"
    assert by_name["A ray.remote"]  # the actor creation call


def test_tracing_off_records_nothing(tmp_path):
    if ray.is_initialized():
        ray.shutdown()
    tracing.disable()
    ray.init(num_cpus=1)
    try:
        @ray.remote
        def f():
            return 1

        assert ray.get(f.remote()) == 1
        assert not tracing.is_enabled()
    finally:
        ray.shutdown()
