"""Declarative Serve config files (reference: python/ray/serve/schema.py ServeDeploySchema /
ServeApplicationSchema / DeploymentSchema, _private/api.py call_app_builder_with_args_if_necessary,
scripts.py ``serve deploy`` / ``serve run`` / ``serve build``).

A config names each application by ``import_path`` (``module:attr`` or ``module.attr``);
the attribute is a bound :class:`Application` or an *app builder* (a function taking the
config's ``args`` dict, or a pydantic model built from it). Per-deployment overrides apply
by deployment name across the whole bound graph, and the application's ``runtime_env``
(``working_dir``/``py_modules``/``env_vars``) is given to every replica so the module that
defines the deployments imports there too.

Deploying a config is declarative: applications in the cluster that the config does not
name are deleted, the rest are (re)deployed with the controller's rolling update."""

from __future__ import annotations

import importlib
import inspect
import json
import os
import sys
from typing import Any, Dict, List, Optional, Union

from pydantic import BaseModel, Field, model_validator

from ray_amd.serve.config import ProxyLocation

_KV_KEY = b"serve:deploy_config"


class DeploymentSchema(BaseModel):
    name: str
    num_replicas: Optional[Union[int, str]] = None
    max_ongoing_requests: Optional[int] = Field(default=None, gt=0)
    max_queued_requests: Optional[int] = None
    user_config: Optional[Any] = None
    autoscaling_config: Optional[Dict[str, Any]] = None
    graceful_shutdown_timeout_s: Optional[float] = Field(default=None, ge=0)
    health_check_period_s: Optional[float] = Field(default=None, gt=0)
    ray_actor_options: Optional[Dict[str, Any]] = None

    @model_validator(mode="after")
    def _check(self):
        if isinstance(self.num_replicas, str) and self.num_replicas != "auto":
            raise ValueError("num_replicas must be an int or 'auto'")
        if self.num_replicas is not None and self.autoscaling_config is not None and \
                self.num_replicas != "auto":
            raise ValueError("num_replicas and autoscaling_config cannot both be set")
        return self

    def overrides(self) -> dict:
        return {k: v for k, v in self.model_dump(exclude_unset=True, exclude_none=True).items()
                if k != "name"}


class ServeApplicationSchema(BaseModel):
    name: str = "default"
    route_prefix: Optional[str] = "/"
    import_path: str
    runtime_env: Dict[str, Any] = Field(default_factory=dict)
    deployments: List[DeploymentSchema] = Field(default_factory=list)
    args: Dict[str, Any] = Field(default_factory=dict)

    @model_validator(mode="after")
    def _check(self):
        if self.route_prefix is not None and not self.route_prefix.startswith("/"):
            raise ValueError(f"route_prefix must start with '/': {self.route_prefix!r}")
        if ":" not in self.import_path and "." not in self.import_path:
            raise ValueError(f"import_path must be 'module:attr' or 'module.attr': "
                             f"{self.import_path!r}")
        names = [d.name for d in self.deployments]
        if len(names) != len(set(names)):
            raise ValueError(f"duplicate deployment names in application {self.name!r}")
        return self


class HTTPOptionsSchema(BaseModel):
    host: str = "127.0.0.1"
    port: int = 8000
    root_path: str = ""
    request_timeout_s: Optional[float] = None
    keep_alive_timeout_s: int = 5


class gRPCOptionsSchema(BaseModel):
    port: int = 9000
    grpc_servicer_functions: List[str] = Field(default_factory=list)


class ServeDeploySchema(BaseModel):
    proxy_location: ProxyLocation = ProxyLocation.EveryNode
    http_options: HTTPOptionsSchema = Field(default_factory=HTTPOptionsSchema)
    grpc_options: gRPCOptionsSchema = Field(default_factory=gRPCOptionsSchema)
    logging_config: Optional[Dict[str, Any]] = None
    applications: List[ServeApplicationSchema] = Field(default_factory=list)

    @model_validator(mode="after")
    def _check(self):
        names = [a.name for a in self.applications]
        if len(names) != len(set(names)):
            raise ValueError(f"application names must be unique: {names}")
        prefixes = [a.route_prefix for a in self.applications if a.route_prefix is not None]
        if len(prefixes) != len(set(prefixes)):
            raise ValueError(f"application route_prefix values must be unique: {prefixes}")
        return self


# ---------------------------------------------------------------- import + build
def _split_import_path(path: str):
    if ":" in path:
        mod, _, attr = path.partition(":")
    else:
        mod, _, attr = path.rpartition(".")
    if not mod or not attr:
        raise ValueError(f"bad import_path {path!r}")
    return mod, attr


def import_attr(path: str, working_dir: Optional[str] = None):
    mod, attr = _split_import_path(path)
    if working_dir and os.path.isdir(working_dir) and working_dir not in sys.path:
        sys.path.insert(0, working_dir)
    obj = importlib.import_module(mod)
    for part in attr.split("."):
        obj = getattr(obj, part)
    return obj


def call_app_builder(target, args: dict):
    """An Application as is (no args allowed), or a builder called with ``args`` (as a
    pydantic model when the builder's single parameter is annotated with one)."""
    from ray_amd.serve.api import Application, Deployment

    if isinstance(target, Deployment):
        target = target.bind()
    if isinstance(target, Application):
        if args:
            raise ValueError("args were given but the import path is an Application, not an "
                             "application builder")
        return target
    if not callable(target):
        raise TypeError(f"import path resolved to {target!r}: expected an Application or a "
                        f"builder function")
    params = list(inspect.signature(target).parameters.values())
    arg = args
    if params:
        ann = params[0].annotation
        if isinstance(ann, str):
            ann = getattr(sys.modules.get(target.__module__), ann, ann)
        if inspect.isclass(ann) and issubclass(ann, BaseModel):
            arg = ann(**args)
        app = target(arg)
    else:
        if args:
            raise ValueError("args were given but the app builder takes no parameters")
        app = target()
    if isinstance(app, Deployment):
        app = app.bind()
    if not isinstance(app, Application):
        raise TypeError(f"app builder {target.__name__} returned {type(app).__name__}, "
                        f"not an Application")
    return app


def apply_overrides(app, overrides: Dict[str, dict], runtime_env: Optional[dict] = None):
    """Copy of the bound graph with per-deployment option overrides (by name) and the
    application runtime_env merged into every deployment's ray_actor_options."""
    from ray_amd.serve.api import Application

    unknown = set(overrides)
    memo: dict = {}

    def conv(v):
        if isinstance(v, Application):
            return rebuild(v)
        if isinstance(v, (list, tuple)):
            return type(v)(conv(x) for x in v)
        if isinstance(v, dict):
            return {k: conv(x) for k, x in v.items()}
        return v

    def rebuild(a):
        if id(a) in memo:
            return memo[id(a)]
        dep = a.deployment
        kw = dict(overrides.get(dep.name, {}))
        unknown.discard(dep.name)
        if kw.get("num_replicas") == "auto" or "autoscaling_config" in kw:
            kw.setdefault("num_replicas", 1)
        if runtime_env:
            opts = dict(kw.get("ray_actor_options", dep.ray_actor_options) or {})
            env = dict(runtime_env)
            env.update(opts.get("runtime_env") or {})
            opts["runtime_env"] = env
            kw["ray_actor_options"] = opts
        new = Application(dep.options(**kw) if kw else dep, conv(a.args), conv(a.kwargs))
        memo[id(a)] = new
        return new

    out = rebuild(app)
    if unknown:
        raise ValueError(f"config names deployments that are not in the application: "
                         f"{sorted(unknown)}")
    return out


def build_application(app_cfg: ServeApplicationSchema):
    wd = app_cfg.runtime_env.get("working_dir")
    target = import_attr(app_cfg.import_path, wd)
    app = call_app_builder(target, app_cfg.args)
    return apply_overrides(app, {d.name: d.overrides() for d in app_cfg.deployments},
                           app_cfg.runtime_env or None)


def deploy_config(config) -> Dict[str, Any]:
    """Deploy a ServeDeploySchema (or its dict / YAML path) declaratively."""
    from ray_amd import serve
    from ray_amd.experimental import internal_kv
    from ray_amd.serve.api import HTTPOptions

    if isinstance(config, str):
        config = load_config_file(config)
    if isinstance(config, dict):
        config = ServeDeploySchema(**config)
    ho = config.http_options
    http = HTTPOptions(host=ho.host, port=ho.port, root_path=ho.root_path,
                       location={ProxyLocation.Disabled: "NoServer",
                                 ProxyLocation.EveryNode: "EveryNode"}.get(
                           ProxyLocation(config.proxy_location), "HeadOnly"))
    grpc = None
    if config.grpc_options.grpc_servicer_functions:
        grpc = {"port": config.grpc_options.port,
                "grpc_servicer_functions": config.grpc_options.grpc_servicer_functions}
    serve.start(http_options=http, grpc_options=grpc)
    handles = {}
    wanted = {a.name for a in config.applications}
    for name in list(serve.status()):
        if name not in wanted:
            serve.delete(name)
    for app_cfg in config.applications:
        app = build_application(app_cfg)
        handles[app_cfg.name] = serve.run(app, name=app_cfg.name,
                                          route_prefix=app_cfg.route_prefix)
    internal_kv._internal_kv_put(_KV_KEY, json.dumps(config.model_dump(mode="json")).encode(),
                                 overwrite=True, namespace="serve")
    return handles


def get_deployed_config() -> Optional[dict]:
    from ray_amd.experimental import internal_kv

    raw = internal_kv._internal_kv_get(_KV_KEY, namespace="serve")
    return json.loads(raw) if raw else None


def load_config_file(path: str) -> ServeDeploySchema:
    import yaml

    with open(path) as f:
        data = yaml.safe_load(f) or {}
    if "applications" not in data and "import_path" in data:
        data = {"applications": [data]}  # a single-application config file
    return ServeDeploySchema(**data)


def build_config(import_path: str, *, name: str = "default", route_prefix: str = "/",
                 working_dir: Optional[str] = None) -> dict:
    """``serve build``: a config file body listing every deployment of the bound graph with
    its current options (edit it, then ``serve deploy`` it)."""
    from ray_amd.serve.api import Application

    app = call_app_builder(import_attr(import_path, working_dir), {})
    deps, seen = [], set()

    def walk(v):
        if isinstance(v, Application):
            d = v.deployment
            for x in list(v.args) + list(v.kwargs.values()):
                walk(x)
            if d.name not in seen:
                seen.add(d.name)
                e = {"name": d.name, "max_ongoing_requests": d.max_ongoing_requests}
                if d.autoscaling_config:
                    e["autoscaling_config"] = d.autoscaling_config
                else:
                    e["num_replicas"] = d.num_replicas
                if d.user_config is not None:
                    e["user_config"] = d.user_config
                if d.ray_actor_options:
                    e["ray_actor_options"] = d.ray_actor_options
                if d.max_queued_requests != -1:
                    e["max_queued_requests"] = d.max_queued_requests
                deps.append(e)
        elif isinstance(v, (list, tuple)):
            for x in v:
                walk(x)
        elif isinstance(v, dict):
            for x in v.values():
                walk(x)

    walk(app)
    app_entry = {"name": name, "route_prefix": route_prefix, "import_path": import_path,
                 "runtime_env": {"working_dir": working_dir} if working_dir else {},
                 "deployments": deps}
    return ServeDeploySchema(applications=[app_entry]).model_dump(mode="json", exclude_none=True)
