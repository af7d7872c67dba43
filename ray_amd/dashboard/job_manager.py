"""Job submission backend: one detached supervisor actor per submitted job.

Parity with ``python/ray/dashboard/modules/job/job_manager.py`` (JobManager.submit_job /
stop_job / get_job_logs / list_jobs; JobSupervisor actor running the entrypoint as a
child process, status PENDING → RUNNING → SUCCEEDED/FAILED/STOPPED kept in the GCS KV).

The supervisor reserves the job's ``entrypoint_num_cpus/_gpus/_resources`` (so a GPU
entrypoint gets its HIP_VISIBLE_DEVICES from the scheduler like any GPU actor), starts
``bash -c <entrypoint>`` in its own process group with ``RAY_ADDRESS`` pointing at this
cluster, tees stdout/stderr into ``<session>/logs/job-driver-<id>.log`` and records the
exit status. Job records live in the internal KV (namespace ``job``) so any driver or
the HTTP head can read them.
"""

from __future__ import annotations

import json
import os
import signal
import subprocess
import threading
import time
import uuid
from enum import Enum
from typing import Any, Dict, Optional

import ray_amd as ray
from ray_amd.experimental import internal_kv as kv

KV_NS = "job"
SUPERVISOR_NS = "_ray_internal_jobs"


class JobStatus(str, Enum):
    PENDING = "PENDING"
    RUNNING = "RUNNING"
    STOPPED = "STOPPED"
    SUCCEEDED = "SUCCEEDED"
    FAILED = "FAILED"

    def __str__(self):
        return self.value

    def is_terminal(self) -> bool:
        return self in (JobStatus.STOPPED, JobStatus.SUCCEEDED, JobStatus.FAILED)


def _key(job_id: str) -> str:
    return f"job_info:{job_id}"


def get_info(job_id: str) -> Optional[dict]:
    raw = kv._internal_kv_get(_key(job_id), namespace=KV_NS)
    return None if raw is None else json.loads(raw)


def _put_info(info: dict) -> None:
    kv._internal_kv_put(_key(info["submission_id"]), json.dumps(info).encode(), namespace=KV_NS)


def _update(job_id: str, **fields) -> dict:
    info = get_info(job_id) or {}
    if info.get("status") in ("STOPPED",) and fields.get("status") in ("SUCCEEDED", "FAILED"):
        fields.pop("status")  # a stop wins over the exit status it caused
        fields.pop("message", None)
    info.update(fields)
    _put_info(info)
    return info


def log_path(session_dir: str, job_id: str) -> str:
    return os.path.join(session_dir, "logs", f"job-driver-{job_id}.log")


@ray.remote(max_concurrency=4)
class JobSupervisor:
    def __init__(self, job_id: str, entrypoint: str, session_dir: str, runtime_env: dict):
        self.job_id = job_id
        self.entrypoint = entrypoint
        self.session_dir = session_dir
        self.runtime_env = runtime_env or {}
        self.proc: Optional[subprocess.Popen] = None
        self.stopped = False

    def run(self) -> int:
        os.makedirs(os.path.join(self.session_dir, "logs"), exist_ok=True)
        env = dict(os.environ)
        env["RAY_ADDRESS"] = self.session_dir
        env["RAY_JOB_SUBMISSION_ID"] = self.job_id
        env.update({k: str(v) for k, v in (self.runtime_env.get("env_vars") or {}).items()})
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH")
                                        else "")
        cwd = self.runtime_env.get("working_dir") or os.getcwd()
        path = log_path(self.session_dir, self.job_id)
        with open(path, "ab", buffering=0) as logf:
            self.proc = subprocess.Popen(["bash", "-c", self.entrypoint], stdout=logf,
                                         stderr=subprocess.STDOUT, cwd=cwd, env=env,
                                         start_new_session=True)
            _update(self.job_id, status="RUNNING", start_time=int(time.time() * 1000),
                    driver_pid=self.proc.pid)
            rc = self.proc.wait()
        if self.stopped:
            _update(self.job_id, status="STOPPED", end_time=int(time.time() * 1000),
                    driver_exit_code=rc, message="Job was intentionally stopped.")
        elif rc == 0:
            _update(self.job_id, status="SUCCEEDED", end_time=int(time.time() * 1000),
                    driver_exit_code=0, message="Job finished successfully.")
        else:
            _update(self.job_id, status="FAILED", end_time=int(time.time() * 1000),
                    driver_exit_code=rc, error_type="JOB_ENTRYPOINT_COMMAND_ERROR",
                    message=f"Job entrypoint command failed with exit code {rc}.")
        return rc

    def stop(self, grace_s: float = 3.0) -> bool:
        self.stopped = True
        _update(self.job_id, status="STOPPED")
        p = self.proc
        if p is None or p.poll() is not None:
            return p is not None
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            return True
        t0 = time.time()
        while p.poll() is None and time.time() - t0 < grace_s:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        return True


class JobManager:
    """Used by the HTTP head (and usable from any connected driver)."""

    def __init__(self, session_dir: Optional[str] = None):
        from ray_amd._private import worker as _w

        self.session_dir = session_dir or _w.global_worker.session_dir
        self._runs: Dict[str, Any] = {}
        self._lock = threading.Lock()

    def submit_job(self, *, entrypoint: str, submission_id: Optional[str] = None,
                   runtime_env: Optional[dict] = None, metadata: Optional[dict] = None,
                   entrypoint_num_cpus=None, entrypoint_num_gpus=None,
                   entrypoint_memory=None, entrypoint_resources=None) -> str:
        job_id = submission_id or f"raysubmit_{uuid.uuid4().hex[:16]}"
        if get_info(job_id) is not None:
            raise ValueError(f"Job with submission_id {job_id} already exists. "
                             "Please use a different submission_id.")
        info = {"submission_id": job_id, "job_id": None, "type": "SUBMISSION",
                "entrypoint": entrypoint, "status": "PENDING", "message": "Job is pending.",
                "metadata": metadata or {}, "runtime_env": runtime_env or {},
                "entrypoint_num_cpus": entrypoint_num_cpus,
                "entrypoint_num_gpus": entrypoint_num_gpus,
                "entrypoint_memory": entrypoint_memory,
                "entrypoint_resources": entrypoint_resources, "start_time": None,
                "end_time": None, "error_type": None, "driver_exit_code": None,
                "driver_node_id": None}
        _put_info(info)
        opts = {"name": f"_ray_internal_job_actor_{job_id}", "namespace": SUPERVISOR_NS,
                "lifetime": "detached", "num_cpus": entrypoint_num_cpus or 0}
        if entrypoint_num_gpus:
            opts["num_gpus"] = entrypoint_num_gpus
        if entrypoint_resources:
            opts["resources"] = entrypoint_resources
        if entrypoint_memory:
            opts["memory"] = entrypoint_memory
        try:
            sup = JobSupervisor.options(**opts).remote(job_id, entrypoint, self.session_dir,
                                                       runtime_env or {})
            ref = sup.run.remote()
        except Exception as e:  # noqa: BLE001
            _update(job_id, status="FAILED", error_type="JOB_SUPERVISOR_ACTOR_START_FAILURE",
                    message=f"Failed to start the job supervisor: {e!r}")
            return job_id
        with self._lock:
            self._runs[job_id] = (sup, ref)
        return job_id

    def _supervisor(self, job_id):
        with self._lock:
            r = self._runs.get(job_id)
        if r is not None:
            return r[0]
        try:
            return ray.get_actor(f"_ray_internal_job_actor_{job_id}", namespace=SUPERVISOR_NS)
        except Exception:
            return None

    def stop_job(self, job_id: str) -> bool:
        info = get_info(job_id)
        if info is None:
            raise ValueError(f"Job {job_id} does not exist.")
        if JobStatus(info["status"]).is_terminal():
            return False
        sup = self._supervisor(job_id)
        if sup is None:
            _update(job_id, status="STOPPED", end_time=int(time.time() * 1000))
            return True
        return bool(ray.get(sup.stop.remote()))

    def delete_job(self, job_id: str) -> bool:
        info = get_info(job_id)
        if info is None:
            raise ValueError(f"Job {job_id} does not exist.")
        if not JobStatus(info["status"]).is_terminal():
            raise RuntimeError(f"Attempted to delete job '{job_id}', but it is in a "
                               f"non-terminal state {info['status']}.")
        kv._internal_kv_del(_key(job_id), namespace=KV_NS)
        sup = self._supervisor(job_id)
        if sup is not None:
            try:
                ray.kill(sup)
            except Exception:
                pass
        with self._lock:
            self._runs.pop(job_id, None)
        return True

    def get_job_info(self, job_id: str) -> Optional[dict]:
        return get_info(job_id)

    def list_jobs(self) -> Dict[str, dict]:
        out = {}
        for k in kv._internal_kv_list("job_info:", namespace=KV_NS):
            k = k.decode() if isinstance(k, bytes) else k
            jid = k.split(":", 1)[1]
            info = get_info(jid)
            if info is not None:
                out[jid] = info
        return out

    def get_job_logs(self, job_id: str) -> str:
        try:
            with open(log_path(self.session_dir, job_id), "rb") as f:
                return f.read().decode(errors="replace")
        except FileNotFoundError:
            return ""
