"""JobConfig (modelled on python/ray/tests/test_job.py / test_runtime_env.py job-level
cases): runtime_env, namespace, code_search_path, metadata and default actor lifetime
given to ray.init through a JobConfig; ray.types / util.serialization modules."""

import os
import tempfile

import pytest

import ray_amd as ray
from ray_amd.job_config import JobConfig


def test_job_config_validation():
    with pytest.raises(ValueError):
        JobConfig(default_actor_lifetime="forever")
    jc = JobConfig(metadata={"a": "1"}, ray_namespace="ns")
    jc.set_metadata("b", "2")
    back = JobConfig.from_json(jc._serialize())
    assert back.metadata == {"a": "1", "b": "2"} and back.ray_namespace == "ns"


def test_job_config_applies_to_the_job():
    d = tempfile.mkdtemp(prefix="jcpath")
    with open(os.path.join(d, "jc_helper_mod.py"), "w") as f:
        f.write("def value():\n    return 'from-code-search-path'\n")
    jc = JobConfig(runtime_env={"env_vars": {"JC_TEST_VAR": "seven"}},
                   metadata={"owner": "tests"}, ray_namespace="jc_ns",
                   code_search_path=[d], default_actor_lifetime="detached")
    ray.init(num_cpus=2, job_config=jc)
    try:
        @ray.remote
        def probe():
            import jc_helper_mod

            return os.environ.get("JC_TEST_VAR"), jc_helper_mod.value()

        assert ray.get(probe.remote()) == ("seven", "from-code-search-path")
        assert ray.get_runtime_context().namespace == "jc_ns"

        @ray.remote
        class A:
            def ping(self):
                return "pong"

        a = A.remote()
        b = A.options(lifetime="non_detached").remote()
        assert ray.get([a.ping.remote(), b.ping.remote()]) == ["pong", "pong"]
        from ray_amd.util.state import list_actors, list_jobs

        det = {r["actor_id"]: r["is_detached"] for r in list_actors()}
        assert sorted(det.values()) == [False, True]
        jobs = list_jobs()
        assert any(j["metadata"] == {"owner": "tests"} for j in jobs)
        ray.kill(a)
    finally:
        ray.shutdown()


def test_types_and_serialization_modules():
    from ray_amd.types import ObjectRef
    from ray_amd.util.check_serialize import inspect_serializability
    from ray_amd.util.serialization import deregister_serializer, register_serializer

    def annotated(x: ObjectRef[int]) -> ObjectRef[str]:
        return x

    assert annotated.__annotations__["x"] is ObjectRef
    assert callable(register_serializer) and callable(deregister_serializer)
    ok, _ = inspect_serializability(lambda: 1, name="fn")
    assert ok


def test_runtime_context_task_names_and_out_of_scope_actor_finishes_calls():
    ray.init(num_cpus=2)
    try:
        @ray.remote
        def my_fn():
            c = ray.get_runtime_context()
            return c.get_task_name(), c.get_task_function_name()

        @ray.remote
        class A:
            def m(self):
                import time

                time.sleep(0.3)
                c = ray.get_runtime_context()
                return c.get_task_name(), c.get_task_function_name()

        name, fq = ray.get(my_fn.remote())
        assert name.endswith("my_fn") and fq.endswith(".my_fn")
        assert ray.get(my_fn.options(name="custom").remote())[0] == "custom"
        # the handle is dropped right after submitting: the call still completes
        name, fq = ray.get(A.remote().m.remote())
        assert name == "A.m" and fq.endswith("A.m")
        assert ray.get_runtime_context().get()["namespace"]
    finally:
        ray.shutdown()
