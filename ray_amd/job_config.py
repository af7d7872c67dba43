"""Per-job driver configuration (reference: python/ray/job_config.py JobConfig).

``ray_amd.init(job_config=JobConfig(...))`` applies: ``runtime_env`` (the job-level
runtime env every task/actor inherits unless it sets its own), ``ray_namespace``,
``code_search_path`` (directories put on the job's import path in every worker),
``metadata`` (shown by ``util.state.list_jobs``) and ``default_actor_lifetime``
(``"detached"`` makes actors outlive the driver unless they pass ``lifetime=...``).
``jvm_options`` are accepted and ignored: this runtime has no Java workers."""

from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional


class JobConfig:
    def __init__(self, jvm_options: Optional[List[str]] = None,
                 code_search_path: Optional[List[str]] = None,
                 runtime_env: Optional[dict] = None, _client_job: bool = False,
                 metadata: Optional[Dict[str, str]] = None,
                 ray_namespace: Optional[str] = None,
                 default_actor_lifetime: str = "non_detached",
                 _py_driver_sys_path: Optional[List[str]] = None):
        self.jvm_options = list(jvm_options or [])
        self.code_search_path = [os.path.abspath(p) for p in (code_search_path or [])]
        self.metadata: Dict[str, str] = dict(metadata or {})
        self.ray_namespace = ray_namespace
        self._client_job = _client_job
        self._py_driver_sys_path = list(_py_driver_sys_path or [])
        self.set_runtime_env(runtime_env)
        self.set_default_actor_lifetime(default_actor_lifetime)

    def set_metadata(self, key: str, value: str) -> None:
        self.metadata[key] = value

    def set_runtime_env(self, runtime_env: Optional[dict],
                        validate: bool = False) -> None:
        env = dict(runtime_env) if runtime_env is not None else {}
        if validate or env:
            from ray_amd.runtime_env import RuntimeEnv

            RuntimeEnv(**env)  # raises on unknown / malformed fields
        self.runtime_env = env

    def set_ray_namespace(self, ray_namespace: str) -> None:
        self.ray_namespace = ray_namespace

    def set_default_actor_lifetime(self, default_actor_lifetime: str) -> None:
        if default_actor_lifetime not in ("detached", "non_detached"):
            raise ValueError("Default actor lifetime must be one of `detached`, "
                             "`non_detached`")
        self.default_actor_lifetime = default_actor_lifetime

    def _to_dict(self) -> Dict[str, Any]:
        return {"jvm_options": self.jvm_options, "code_search_path": self.code_search_path,
                "runtime_env": self.runtime_env, "metadata": self.metadata,
                "ray_namespace": self.ray_namespace,
                "default_actor_lifetime": self.default_actor_lifetime}

    def _serialize(self) -> str:
        return json.dumps(self._to_dict(), sort_keys=True, default=str)

    @classmethod
    def from_json(cls, job_config_json) -> "JobConfig":
        d = json.loads(job_config_json) if isinstance(job_config_json, str) else \
            dict(job_config_json)
        return cls(**d)

    def __repr__(self):
        return f"JobConfig({self._to_dict()})"
