"""``RuntimeEnv`` / ``RuntimeEnvConfig`` (reference: python/ray/runtime_env/runtime_env.py).

A ``RuntimeEnv`` is a validated dict, so it is accepted anywhere a runtime_env dict is
(``ray_amd.init``, ``.options(runtime_env=...)``, job submission). Fields honoured by this
runtime: ``env_vars``, ``working_dir``, ``py_modules``, ``config``; ``pip`` / ``conda`` /
``uv`` / ``container`` are validated and recorded but cannot install anything offline
(a worker whose env names packages that are not importable fails at setup with
RuntimeEnvSetupError)."""

from __future__ import annotations

from typing import Any, Dict, List, Optional, Union

_KNOWN = ("env_vars", "working_dir", "py_modules", "pip", "conda", "uv", "container",
          "image_uri", "config", "excludes", "py_executable", "java_jars", "_ray_commit",
          "nsight", "mpi", "worker_process_setup_hook")


class RuntimeEnvConfig(dict):
    def __init__(self, setup_timeout_seconds: int = 600, eager_install: bool = True,
                 log_files: Optional[List[str]] = None):
        if not isinstance(setup_timeout_seconds, int) or \
                (setup_timeout_seconds <= 0 and setup_timeout_seconds != -1):
            raise ValueError("setup_timeout_seconds must be a positive int or -1")
        super().__init__(setup_timeout_seconds=setup_timeout_seconds,
                         eager_install=bool(eager_install), log_files=list(log_files or []))

    @staticmethod
    def parse_and_validate_runtime_env_config(config) -> "RuntimeEnvConfig":
        if isinstance(config, RuntimeEnvConfig):
            return config
        if isinstance(config, dict):
            return RuntimeEnvConfig(**config)
        raise TypeError(f"config must be a dict or RuntimeEnvConfig, got {type(config)}")


class RuntimeEnv(dict):
    def __init__(self, *, py_modules: Optional[List[str]] = None,
                 working_dir: Optional[str] = None,
                 pip: Optional[Union[List[str], str, Dict]] = None,
                 conda: Optional[Union[Dict[str, str], str]] = None,
                 container: Optional[Dict[str, str]] = None,
                 env_vars: Optional[Dict[str, str]] = None,
                 config: Optional[Union[Dict, RuntimeEnvConfig]] = None,
                 _validate: bool = True, **kwargs):
        super().__init__()
        fields = dict(py_modules=py_modules, working_dir=working_dir, pip=pip, conda=conda,
                      container=container, env_vars=env_vars, config=config, **kwargs)
        for k, v in fields.items():
            if v is not None:
                self[k] = v
        if _validate:
            self._validate()

    def _validate(self):
        unknown = [k for k in self if k not in _KNOWN]
        if unknown:
            raise ValueError(f"unknown runtime_env fields {unknown}; known: {list(_KNOWN)}")
        ev = self.get("env_vars")
        if ev is not None and not (isinstance(ev, dict) and all(
                isinstance(k, str) and isinstance(v, str) for k, v in ev.items())):
            raise TypeError("runtime_env['env_vars'] must be a Dict[str, str]")
        if "pip" in self and "conda" in self:
            raise ValueError("The 'pip' field and 'conda' field of runtime_env cannot both "
                             "be specified.")
        wd = self.get("working_dir")
        if wd is not None and not isinstance(wd, str):
            raise TypeError("runtime_env['working_dir'] must be a str")
        pm = self.get("py_modules")
        if pm is not None and not isinstance(pm, list):
            raise TypeError("runtime_env['py_modules'] must be a list")
        if "config" in self:
            self["config"] = RuntimeEnvConfig.parse_and_validate_runtime_env_config(
                self["config"])

    def to_dict(self) -> Dict[str, Any]:
        return dict(self)

    @classmethod
    def deserialize(cls, serialized: str) -> "RuntimeEnv":
        import json

        return cls(**json.loads(serialized))

    def serialize(self) -> str:
        import json

        return json.dumps(self, sort_keys=True)

    def env_vars(self) -> Dict[str, str]:
        return dict(self.get("env_vars") or {})

    def working_dir_uri(self) -> Optional[str]:
        return self.get("working_dir")

    def py_modules_uris(self) -> List[str]:
        return list(self.get("py_modules") or [])

    def has_py_container(self) -> bool:
        return "container" in self


__all__ = ["RuntimeEnv", "RuntimeEnvConfig"]
