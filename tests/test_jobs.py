"""Job submission, HTTP head and CLI tests (modelled on dashboard/modules/job/tests/
test_job_manager.py + test_sdk.py, and python/ray/tests/test_cli.py)."""

import json
import os
import socket
import subprocess
import sys
import textwrap
import urllib.request

import pytest

import ray_amd as ray
from ray_amd.job_submission import JobStatus, JobSubmissionClient

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def head():
    ctx = ray.init(num_cpus=4, include_dashboard=True, dashboard_port=_free_port())
    yield ctx
    ray.shutdown()


TERMINAL = {JobStatus.SUCCEEDED, JobStatus.FAILED, JobStatus.STOPPED}


def test_submit_success_and_logs(head, tmp_path):
    (tmp_path / "job.py").write_text(textwrap.dedent("""
        import os
        import ray_amd as ray
        ray.init()
        @ray.remote
        def sq(x):
            return x * x
        print("answer", sum(ray.get([sq.remote(i) for i in range(5)])), os.environ["MY_VAR"])
    """))
    c = JobSubmissionClient(head.dashboard_url)
    jid = c.submit_job(entrypoint=f"{sys.executable} job.py", submission_id="job_ok",
                       runtime_env={"working_dir": str(tmp_path), "env_vars": {"MY_VAR": "hi"}},
                       metadata={"owner": "test"})
    assert jid == "job_ok"
    assert c.wait_until_status(jid, TERMINAL, 120) == JobStatus.SUCCEEDED
    assert "answer 30 hi" in c.get_job_logs(jid)
    info = c.get_job_info(jid)
    assert info.metadata == {"owner": "test"} and info.driver_exit_code == 0
    assert info.start_time <= info.end_time
    with pytest.raises(RuntimeError):
        c.submit_job(entrypoint="true", submission_id="job_ok")  # duplicate id


def test_failed_and_stopped_jobs(head):
    c = JobSubmissionClient(head.dashboard_url)
    bad = c.submit_job(entrypoint="echo oops; exit 3")
    assert c.wait_until_status(bad, TERMINAL, 60) == JobStatus.FAILED
    assert c.get_job_info(bad).driver_exit_code == 3
    assert "oops" in c.get_job_logs(bad)
    slow = c.submit_job(entrypoint="sleep 600", entrypoint_num_cpus=1)
    c.wait_until_status(slow, {JobStatus.RUNNING}, 60)
    assert c.stop_job(slow) is True
    assert c.wait_until_status(slow, TERMINAL, 30) == JobStatus.STOPPED
    ids = {j.submission_id for j in c.list_jobs()}
    assert {bad, slow} <= ids
    assert c.delete_job(bad) is True
    assert bad not in {j.submission_id for j in c.list_jobs()}


def test_http_state_and_metrics(head):
    url = head.dashboard_url
    with urllib.request.urlopen(url + "/api/v0/nodes") as r:
        body = json.loads(r.read())
    assert body["result"] and body["data"]["result"]["total"] == 1
    with urllib.request.urlopen(url + "/api/v0/tasks/summarize") as r:
        assert "cluster" in json.loads(r.read())["data"]["result"]
    with urllib.request.urlopen(url + "/api/cluster_status") as r:
        assert json.loads(r.read())["data"]["clusterStatus"]["totalResources"]["CPU"] == 4
    with urllib.request.urlopen(url + "/metrics") as r:
        assert b"ray_object_store_memory" in r.read()


def test_cli_start_status_stop():
    import pathlib
    import shutil
    import tempfile

    tmp_path = pathlib.Path(tempfile.mkdtemp(prefix="racli", dir="/tmp"))  # short: unix sockets
    env = dict(os.environ, RAY_AMD_TMPDIR=str(tmp_path), PYTHONPATH=REPO)
    env.pop("RAY_ADDRESS", None)

    def run(*args, timeout=120):
        return subprocess.run([sys.executable, "-m", "ray_amd.scripts", *args], env=env,
                              cwd=str(tmp_path), capture_output=True, text=True,
                              timeout=timeout, stdin=subprocess.DEVNULL)

    r = run("start", "--head", "--num-cpus", "2", "--dashboard-port", str(_free_port()))
    assert r.returncode == 0, r.stderr
    try:
        r = run("status")
        assert r.returncode == 0 and "0/2 CPU" in r.stdout, r.stdout + r.stderr
        r = run("job", "submit", "--", "echo", "from-job")
        assert r.returncode == 0 and "from-job" in r.stdout, r.stdout + r.stderr
        r = run("list", "jobs", "--format", "json")
        assert r.returncode == 0 and json.loads(r.stdout), r.stderr
        r = run("summary", "tasks")
        assert r.returncode == 0 and "cluster" in json.loads(r.stdout)
        r = run("start", "--address", "auto", "--num-cpus", "3")  # join a worker node
        assert r.returncode == 0, r.stderr
        r = run("status")
        assert r.returncode == 0 and "Nodes: 2 alive" in r.stdout and "0/5 CPU" in r.stdout, \
            r.stdout + r.stderr
    finally:
        r = run("stop")
    assert r.returncode == 0 and "Stopped" in r.stdout
    assert not (tmp_path / "ray_current_cluster").exists()
    shutil.rmtree(tmp_path, ignore_errors=True)
