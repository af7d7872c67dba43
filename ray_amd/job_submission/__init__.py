"""Job submission SDK (parity: ``ray.job_submission`` / dashboard/modules/job/sdk.py:
JobSubmissionClient.submit_job:129, stop_job:257, delete_job:291, get_job_info:328,
list_jobs:362, get_job_status:403, get_job_logs:427, tail_job_logs:456)."""

from __future__ import annotations

import json
import os
import time
import urllib.error
import urllib.request
from dataclasses import dataclass, field
from enum import Enum
from typing import Any, AsyncIterator, Dict, List, Optional

from ray_amd.dashboard.job_manager import JobStatus  # noqa: F401


class JobType(str, Enum):
    """How a job started (reference: dashboard/modules/job/pydantic_models.py:26)."""
    SUBMISSION = "SUBMISSION"  # through the Jobs API
    DRIVER = "DRIVER"  # a driver script that called ray_amd.init


@dataclass
class DriverInfo:
    """The driver process of a job (pydantic_models.py:13)."""
    id: str
    node_ip_address: str
    pid: str


@dataclass
class JobDetails:
    submission_id: str
    entrypoint: str
    status: JobStatus
    type: JobType = JobType.SUBMISSION
    job_id: Optional[str] = None
    message: Optional[str] = None
    error_type: Optional[str] = None
    start_time: Optional[int] = None
    end_time: Optional[int] = None
    metadata: Dict[str, str] = field(default_factory=dict)
    runtime_env: Dict[str, Any] = field(default_factory=dict)
    driver_exit_code: Optional[int] = None
    entrypoint_num_cpus: Optional[float] = None
    entrypoint_num_gpus: Optional[float] = None
    entrypoint_memory: Optional[int] = None
    entrypoint_resources: Optional[Dict[str, float]] = None
    driver_node_id: Optional[str] = None
    driver_pid: Optional[int] = None
    driver_info: Optional[DriverInfo] = None

    @classmethod
    def from_dict(cls, d: dict) -> "JobDetails":
        known = {k: v for k, v in d.items() if k in cls.__dataclass_fields__}
        known["status"] = JobStatus(known["status"])
        known["type"] = JobType(known.get("type") or "SUBMISSION")
        di = known.get("driver_info")
        if isinstance(di, dict):
            known["driver_info"] = DriverInfo(**{k: str(v) for k, v in di.items()
                                                 if k in ("id", "node_ip_address", "pid")})
        elif known.get("driver_pid") is not None and di is None:
            known["driver_info"] = DriverInfo(id=str(known.get("job_id") or ""),
                                              node_ip_address="127.0.0.1",
                                              pid=str(known["driver_pid"]))
        return cls(**known)


JobInfo = JobDetails


def _resolve_address(address: Optional[str]) -> str:
    if address is None:
        address = os.environ.get("RAY_AMD_DASHBOARD_ADDRESS") or os.environ.get("RAY_ADDRESS")
    if address in (None, "auto") or (address and not address.startswith("http")):
        from ray_amd._private.worker import CURRENT_CLUSTER_FILE

        session = address if address not in (None, "auto") else None
        if session is None and os.path.exists(CURRENT_CLUSTER_FILE):
            with open(CURRENT_CLUSTER_FILE) as f:
                session = f.read().strip()
        if session and os.path.exists(os.path.join(session, "dashboard.json")):
            with open(os.path.join(session, "dashboard.json")) as f:
                return json.load(f)["url"]
        return "http://127.0.0.1:8265"
    return address.rstrip("/")


class JobSubmissionClient:
    def __init__(self, address: Optional[str] = None, headers: Optional[dict] = None,
                 verify=True, **kw):
        self._address = _resolve_address(address)
        self._headers = headers or {}
        self._request("GET", "/api/version")  # fail fast, like the reference

    def _request(self, method: str, path: str, body: Optional[dict] = None, raw=False):
        data = None if body is None else json.dumps(body).encode()
        req = urllib.request.Request(self._address + path, data=data, method=method,
                                     headers={"Content-Type": "application/json",
                                              **self._headers})
        try:
            with urllib.request.urlopen(req, timeout=60) as r:
                payload = r.read()
        except urllib.error.HTTPError as e:
            msg = e.read().decode(errors="replace")
            if e.code == 404:
                raise RuntimeError(f"Request failed with status code 404: {msg}") from None
            raise RuntimeError(f"Request failed with status code {e.code}: {msg}") from None
        except urllib.error.URLError as e:
            raise ConnectionError(f"Failed to connect to the job server at {self._address}: "
                                  f"{e.reason}") from None
        return payload if raw else json.loads(payload)

    def submit_job(self, *, entrypoint: str, job_id: Optional[str] = None,
                   runtime_env: Optional[Dict[str, Any]] = None,
                   metadata: Optional[Dict[str, str]] = None, submission_id: Optional[str] = None,
                   entrypoint_num_cpus=None, entrypoint_num_gpus=None, entrypoint_memory=None,
                   entrypoint_resources=None) -> str:
        runtime_env = dict(runtime_env or {})
        if runtime_env.get("working_dir"):
            runtime_env["working_dir"] = os.path.abspath(runtime_env["working_dir"])
        r = self._request("POST", "/api/jobs/", {
            "entrypoint": entrypoint, "submission_id": submission_id or job_id,
            "runtime_env": runtime_env, "metadata": metadata or {},
            "entrypoint_num_cpus": entrypoint_num_cpus,
            "entrypoint_num_gpus": entrypoint_num_gpus, "entrypoint_memory": entrypoint_memory,
            "entrypoint_resources": entrypoint_resources})
        return r["submission_id"]

    def stop_job(self, job_id: str) -> bool:
        return self._request("POST", f"/api/jobs/{job_id}/stop", {})["stopped"]

    def delete_job(self, job_id: str) -> bool:
        return self._request("DELETE", f"/api/jobs/{job_id}")["deleted"]

    def get_job_info(self, job_id: str) -> JobDetails:
        return JobDetails.from_dict(self._request("GET", f"/api/jobs/{job_id}"))

    def list_jobs(self) -> List[JobDetails]:
        return [JobDetails.from_dict(d) for d in self._request("GET", "/api/jobs/")]

    def get_job_status(self, job_id: str) -> JobStatus:
        return self.get_job_info(job_id).status

    def get_job_logs(self, job_id: str) -> str:
        return self._request("GET", f"/api/jobs/{job_id}/logs")["logs"]

    async def tail_job_logs(self, job_id: str) -> AsyncIterator[str]:
        import asyncio

        loop = asyncio.get_running_loop()
        req = urllib.request.Request(self._address + f"/api/jobs/{job_id}/logs/tail")
        resp = await loop.run_in_executor(None, lambda: urllib.request.urlopen(req, timeout=3600))
        try:
            while True:
                chunk = await loop.run_in_executor(None, lambda: resp.read1(65536))
                if not chunk:
                    return
                yield chunk.decode(errors="replace")
        finally:
            resp.close()

    def wait_until_status(self, job_id: str, statuses, timeout_s: float = 60.0) -> JobStatus:
        t0 = time.time()
        while True:
            s = self.get_job_status(job_id)
            if s in statuses:
                return s
            if time.time() - t0 > timeout_s:
                raise TimeoutError(f"job {job_id} still {s} after {timeout_s}s")
            time.sleep(0.1)


__all__ = ["JobSubmissionClient", "JobStatus", "JobDetails", "JobInfo", "JobType", "DriverInfo"]
