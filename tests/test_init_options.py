"""ray_amd.init options honoured or rejected (reference: ray.init): unknown keywords raise,
_system_config keys map onto the raylet's RAY_<key> settings (unknown keys raise),
log_to_driver=False keeps worker output out of the driver terminal (it still lands in the
per-worker log files), storage sets the default results storage, logging_level is applied."""
import glob
import logging
import os
import subprocess
import sys
import textwrap

import pytest

import ray_amd as ray


def test_unknown_keyword_and_system_config_validation():
    with pytest.raises(TypeError, match="unexpected keyword"):
        ray.init(num_cpus=1, no_such_option=1)
    with pytest.raises(ValueError, match="unsupported _system_config key"):
        ray.init(num_cpus=1, _system_config={"made_up": 1})
    assert not ray.is_initialized()


def _run(code):
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], capture_output=True,
                          text=True, timeout=120, cwd=os.getcwd(),
                          env=dict(os.environ, PYTHONPATH=os.getcwd()))


def test_log_to_driver_false_and_system_config(tmp_path):
    code = f"""
    import glob, os, time, logging
    import ray_amd as ray
    ctx = ray.init(num_cpus=1, log_to_driver=False, logging_level=logging.DEBUG,
                   storage={str(tmp_path)!r},
                   _system_config={{"memory_usage_threshold": 0.99}})

    @ray.remote
    def hello():
        print("WORKER-SAYS-HI", flush=True)
        return os.environ.get("RAY_memory_usage_threshold")

    print("threshold", ray.get(hello.remote()))
    print("level", logging.getLogger("ray_amd").level)
    print("storage", os.environ.get("RAY_AMD_STORAGE"))
    time.sleep(0.5)
    logs = glob.glob(os.path.join(ctx["session_dir"], "logs", "worker-*.out"))
    print("in_files", any("WORKER-SAYS-HI" in open(p).read() for p in logs))
    ray.shutdown()
    """
    r = _run(code)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "WORKER-SAYS-HI" not in r.stdout.replace("in_files", "")
    assert "threshold 0.99" in r.stdout  # the raylet (and its workers) got RAY_<key>
    assert f"level {logging.DEBUG}" in r.stdout
    assert f"storage {tmp_path}" in r.stdout
    assert "in_files True" in r.stdout
