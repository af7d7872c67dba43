"""worker_process_setup_hook and unhandled-error reporting (modelled on
python/ray/tests/test_runtime_env_setup_func.py and test_unhandled_error.py)."""

import os
import subprocess
import sys
import textwrap

import pytest

import ray_amd as ray
from ray_amd.exceptions import RuntimeEnvSetupError

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _hook():
    import logging

    os.environ["SETUP_HOOK_RAN"] = "1"
    logging.getLogger("setup_hook_test").setLevel(logging.DEBUG)


def _bad_hook():
    raise ValueError("hook exploded")


def test_setup_hook_callable_job_level_and_task_level():
    ray.init(num_cpus=2, runtime_env={"worker_process_setup_hook": _hook})
    try:
        @ray.remote
        def probe():
            import logging

            return (os.environ.get("SETUP_HOOK_RAN"),
                    logging.getLogger("setup_hook_test").level)

        assert ray.get(probe.remote()) == ("1", 10)

        @ray.remote
        class A:
            def probe(self):
                return os.environ.get("SETUP_HOOK_RAN")

        assert ray.get(A.remote().probe.remote()) == "1"

        @ray.remote(runtime_env={"worker_process_setup_hook": _bad_hook})
        def doomed():
            return 1

        with pytest.raises(RuntimeEnvSetupError, match="hook exploded"):
            ray.get(doomed.remote())
    finally:
        ray.shutdown()


def test_setup_hook_import_path(tmp_path):
    (tmp_path / "hookmod.py").write_text(
        "import os\ndef setup():\n    os.environ['HOOK_FROM_PATH'] = 'yes'\n")
    ray.init(num_cpus=2, runtime_env={"worker_process_setup_hook": "hookmod.setup",
                                      "py_modules": [str(tmp_path)]})
    try:
        @ray.remote
        def probe():
            return os.environ.get("HOOK_FROM_PATH")

        assert ray.get(probe.remote()) == "yes"
    finally:
        ray.shutdown()


def _run_driver(body: str, env=None):
    code = textwrap.dedent('''
        import gc, sys, time
        sys.path.insert(0, %r)
        import ray_amd as ray
        ray.init(num_cpus=2)

        @ray.remote
        def f(tag):
            raise ValueError("oops-" + tag)
    ''' % REPO) + textwrap.dedent(body) + "\ntime.sleep(0.5)\nray.shutdown()\n"
    e = dict(os.environ, **(env or {}))
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=120, env=e)


def test_unhandled_error_reported_when_never_read():
    r = _run_driver("""
        r = f.remote("unread")
        ray.wait([r])
        del r
        gc.collect()
    """)
    assert "Unhandled error (suppress with 'RAY_IGNORE_UNHANDLED_ERRORS=1')" in r.stderr
    assert "oops-unread" in r.stderr


def test_read_or_suppressed_errors_are_not_reported():
    r = _run_driver("""
        r = f.remote("read")
        try:
            ray.get(r)
        except Exception:
            pass
        del r
        gc.collect()
    """)
    assert "Unhandled error" not in r.stderr
    r = _run_driver("""
        r = f.remote("quiet")
        ray.wait([r])
        del r
        gc.collect()
    """, env={"RAY_IGNORE_UNHANDLED_ERRORS": "1"})
    assert "Unhandled error" not in r.stderr


def test_actor_death_is_not_an_unhandled_error():
    r = _run_driver("""
        @ray.remote
        class A:
            def slow(self):
                time.sleep(30)

        a = A.remote()
        ref = a.slow.remote()
        time.sleep(0.5)
        ray.kill(a)
        ray.wait([ref], timeout=10)
        del ref
        gc.collect()
    """)
    assert "Unhandled error" not in r.stderr


def test_error_read_by_a_borrower_is_not_reported():
    """The error ref travels inside a list (so it is NOT resolved as an argument) and the
    borrower task ray.get()s it through the owner: the owner must count that as a read."""
    r = _run_driver("""
        @ray.remote
        def reader(lst):
            try:
                ray.get(lst[0])
            except Exception:
                return "seen"

        e = f.remote("borrowed")
        ray.wait([e])
        assert ray.get(reader.remote([e])) == "seen"
        del e
        gc.collect()
    """)
    assert r.returncode == 0, r.stderr
    assert "Unhandled error" not in r.stderr
