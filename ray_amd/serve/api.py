"""Serve public API (reference: python/ray/serve/api.py, deployment.py)."""

from __future__ import annotations

import hashlib
import inspect
import time

import cloudpickle

import ray_amd as ray
from ray_amd.serve._controller import CONTROLLER_NAME, SERVE_NAMESPACE, ServeController
from ray_amd.serve.handle import DeploymentHandle

_controller = None
_proxy = None
_http_port = 8000

try:  # starlette's State recurses in __getattr__ when unpickled: reduce it explicitly
    import copyreg

    from starlette.datastructures import State as _State

    copyreg.pickle(_State, lambda s: (_State, (dict(s._state),)))
except ImportError:  # pragma: no cover
    pass


def _get_controller(create=False):
    global _controller
    if _controller is not None:
        return _controller
    try:
        _controller = ray.get_actor(CONTROLLER_NAME, namespace=SERVE_NAMESPACE)
    except ValueError:
        if not create:
            raise RuntimeError("Serve is not running; call serve.run() or serve.start() first")
        _controller = ray.remote(ServeController).options(
            name=CONTROLLER_NAME, namespace=SERVE_NAMESPACE, lifetime="detached", num_cpus=0,
            max_concurrency=1000, max_restarts=-1, get_if_exists=True).remote()
    return _controller


class HTTPOptions:
    """HTTP proxy settings (reference: serve/config.py HTTPOptions)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 8000, root_path: str = "",
                 location: str = "HeadOnly", request_timeout_s: float | None = None,
                 keep_alive_timeout_s: int = 5, **kw):
        if location not in ("HeadOnly", "EveryNode", "NoServer"):
            raise ValueError(f"invalid HTTP proxy location {location!r}")
        self.host, self.port, self.root_path = host, port, root_path
        self.location = location
        self.request_timeout_s = request_timeout_s
        self.keep_alive_timeout_s = keep_alive_timeout_s

    def to_dict(self) -> dict:
        return dict(self.__dict__)


def start(http_options=None, detached: bool = True, **kw):
    global _proxy, _http_port
    if not ray.is_initialized():
        ray.init()
    c = _get_controller(create=True)
    if isinstance(http_options, HTTPOptions):
        http_options = http_options.to_dict()
    opts = http_options or {}
    port = opts.get("port", 8000)
    existing = ray.get(c.get_proxy.remote())
    if existing is not None and opts and opts != ray.get(c.get_http_options.remote()) and \
            opts.get("location") == "EveryNode":
        ray.get(c.set_proxy.remote(existing, opts))  # switch an existing head proxy's mode
    if existing is None and opts.get("location", "HeadOnly") != "NoServer":
        from ray_amd.serve._proxy import HTTPProxy

        _proxy = ray.remote(HTTPProxy).options(num_cpus=0, max_concurrency=1000,
                                               name="SERVE_PROXY", namespace=SERVE_NAMESPACE,
                                               lifetime="detached").remote(
            opts.get("host", "127.0.0.1"), port, opts.get("request_timeout_s"))
        err = ray.get(_proxy.ping.remote())
        if err != "ok":
            raise RuntimeError(f"HTTP proxy failed to start: {err}")
        ray.get(c.set_proxy.remote(_proxy, opts))
        _http_port = port
    g = kw.get("grpc_options")
    if g is not None:
        g = g if isinstance(g, dict) else vars(g)
        if g.get("grpc_servicer_functions") and ray.get(c.get_grpc_proxy.remote()) is None:
            from ray_amd.serve._grpc_proxy import gRPCProxy

            gp = ray.remote(gRPCProxy).options(
                num_cpus=0, max_concurrency=1000, name="SERVE_GRPC_PROXY",
                namespace=SERVE_NAMESPACE, lifetime="detached").remote(
                g.get("host", "127.0.0.1"), int(g.get("port", 9000)),
                list(g["grpc_servicer_functions"]))
            err = ray.get(gp.ping.remote())
            if err != "ok":
                raise RuntimeError(f"gRPC proxy failed to start: {err}")
            ray.get(c.set_grpc_proxy.remote(gp))
    return c


class gRPCOptions:
    """gRPC ingress options (reference: python/ray/serve/config.py:gRPCOptions)."""

    def __init__(self, port: int = 9000, grpc_servicer_functions=(), host="127.0.0.1"):
        self.port = port
        self.grpc_servicer_functions = list(grpc_servicer_functions)
        self.host = host


def _logging_config(cfg):
    """serve LoggingConfig / dict -> {"log_level": LEVEL}; the replica applies it to its
    Python loggers (reference: serve/schema.py LoggingConfig)."""
    if cfg is None:
        return None
    d = dict(getattr(cfg, "__dict__", cfg)) if not isinstance(cfg, dict) else dict(cfg)
    level = str(d.get("log_level", "INFO")).upper()
    import logging

    if not isinstance(logging.getLevelName(level), int):
        raise ValueError(f"invalid log_level {level!r}")
    unknown = set(d) - {"log_level", "encoding", "logs_dir", "enable_access_log"}
    if unknown:
        raise ValueError(f"unsupported logging_config keys: {sorted(unknown)}")
    return {"log_level": level, "enable_access_log": bool(d.get("enable_access_log", True))}


class Deployment:
    def __init__(self, func_or_class, name, num_replicas=1, ray_actor_options=None,
                 user_config=None, max_ongoing_requests=100, autoscaling_config=None,
                 route_prefix=None, graceful_shutdown_timeout_s=5.0, health_check_period_s=10.0,
                 version=None, max_queued_requests=-1, health_check_timeout_s=30.0,
                 placement_group_bundles=None, placement_group_strategy=None,
                 max_replicas_per_node=None, graceful_shutdown_wait_loop_s=2.0,
                 logging_config=None, **kw):
        from ray_amd.serve.config import normalize_autoscaling_config

        if kw:
            raise TypeError(f"unsupported deployment option(s): {sorted(kw)}")
        if graceful_shutdown_wait_loop_s <= 0:
            raise ValueError("graceful_shutdown_wait_loop_s must be > 0")
        self.graceful_shutdown_wait_loop_s = graceful_shutdown_wait_loop_s
        self.logging_config = _logging_config(logging_config)

        self.func_or_class = func_or_class
        self.name = name
        if num_replicas == "auto":
            autoscaling_config = autoscaling_config or {"min_replicas": 1, "max_replicas": 100,
                                                        "target_ongoing_requests": 2.0}
            num_replicas = 1
        if max_queued_requests != -1 and max_queued_requests < 1:
            raise ValueError("max_queued_requests must be -1 (no limit) or a positive int")
        self.num_replicas = num_replicas
        self.ray_actor_options = ray_actor_options or {}
        self.user_config = user_config
        self.max_ongoing_requests = max_ongoing_requests
        self.max_queued_requests = max_queued_requests
        self.autoscaling_config = normalize_autoscaling_config(autoscaling_config)
        self.route_prefix = route_prefix
        self.graceful_shutdown_timeout_s = graceful_shutdown_timeout_s
        self.health_check_period_s = health_check_period_s
        self.health_check_timeout_s = health_check_timeout_s
        if placement_group_strategy is not None and placement_group_bundles is None:
            raise ValueError("placement_group_strategy needs placement_group_bundles")
        if max_replicas_per_node is not None and placement_group_bundles is not None:
            raise ValueError("max_replicas_per_node cannot be combined with "
                             "placement_group_bundles")
        if max_replicas_per_node is not None and max_replicas_per_node < 1:
            raise ValueError("max_replicas_per_node must be >= 1")
        self.placement_group_bundles = placement_group_bundles
        self.placement_group_strategy = placement_group_strategy
        self.max_replicas_per_node = max_replicas_per_node
        self.version = version

    def options(self, **kw):
        d = dict(num_replicas=self.num_replicas, ray_actor_options=self.ray_actor_options,
                 user_config=self.user_config, max_ongoing_requests=self.max_ongoing_requests,
                 autoscaling_config=self.autoscaling_config, route_prefix=self.route_prefix,
                 graceful_shutdown_timeout_s=self.graceful_shutdown_timeout_s,
                 health_check_period_s=self.health_check_period_s,
                 health_check_timeout_s=self.health_check_timeout_s,
                 placement_group_bundles=self.placement_group_bundles,
                 placement_group_strategy=self.placement_group_strategy,
                 max_replicas_per_node=self.max_replicas_per_node,
                 max_queued_requests=self.max_queued_requests,
                 graceful_shutdown_wait_loop_s=self.graceful_shutdown_wait_loop_s,
                 logging_config=self.logging_config,
                 version=self.version, name=self.name)
        if "max_concurrent_queries" in kw:
            kw["max_ongoing_requests"] = kw.pop("max_concurrent_queries")
        d.update(kw)
        name = d.pop("name")
        return Deployment(self.func_or_class, name, **d)

    def bind(self, *args, **kwargs):
        return Application(self, args, kwargs)

    @property
    def max_concurrent_queries(self) -> int:  # the reference's deprecated name
        return self.max_ongoing_requests

    @property
    def init_args(self) -> tuple:
        return ()

    @property
    def init_kwargs(self) -> dict:
        return {}

    @property
    def url(self):
        """HTTP URL of a deployment with a route prefix (None otherwise)."""
        if self.route_prefix is None:
            return None
        return f"http://127.0.0.1:{_http_port}{self.route_prefix}"

    def set_logging_config(self, logging_config) -> None:
        self.logging_config = _logging_config(logging_config)

    def __call__(self, *a, **k):
        raise RuntimeError("Deployments cannot be constructed directly; use .bind().")


class Application:
    def __init__(self, deployment: Deployment, args, kwargs):
        self.deployment = deployment
        self.args = args
        self.kwargs = kwargs


def deployment(_func_or_class=None, *, name=None, num_replicas=1, ray_actor_options=None,
               user_config=None, max_ongoing_requests=100, max_concurrent_queries=None,
               autoscaling_config=None, route_prefix=None, graceful_shutdown_timeout_s=5.0,
               health_check_period_s=10.0, version=None, max_queued_requests=-1,
               health_check_timeout_s=30.0, placement_group_bundles=None,
               placement_group_strategy=None, max_replicas_per_node=None,
               graceful_shutdown_wait_loop_s=2.0, logging_config=None, **kw):
    if max_concurrent_queries is not None:
        max_ongoing_requests = max_concurrent_queries
    if kw:
        raise TypeError(f"unsupported deployment option(s): {sorted(kw)}")

    def deco(fc):
        return Deployment(fc, name or fc.__name__, num_replicas, ray_actor_options, user_config,
                          max_ongoing_requests, autoscaling_config, route_prefix,
                          graceful_shutdown_timeout_s, health_check_period_s, version,
                          max_queued_requests=max_queued_requests,
                          health_check_timeout_s=health_check_timeout_s,
                          placement_group_bundles=placement_group_bundles,
                          placement_group_strategy=placement_group_strategy,
                          max_replicas_per_node=max_replicas_per_node,
                          graceful_shutdown_wait_loop_s=graceful_shutdown_wait_loop_s,
                          logging_config=logging_config)

    if _func_or_class is not None and callable(_func_or_class):
        return deco(_func_or_class)
    return deco


def ingress(app):
    """Class decorator: serve an ASGI (FastAPI/starlette) app from this deployment."""

    def deco(cls):
        orig_init = cls.__init__

        def __serve_bind_asgi__(self, asgi_app):
            try:
                from fastapi.routing import APIRoute
            except ImportError:
                return
            for route in list(asgi_app.router.routes):
                ep = getattr(route, "endpoint", None)
                if isinstance(route, APIRoute) and ep is not None and \
                        ep.__qualname__.split(".")[-2:] == [cls.__name__, ep.__name__]:
                    # (cloudpickle rebuilds dynamic classes with a bare __qualname__)
                    bound = getattr(self, ep.__name__)
                    asgi_app.router.routes.remove(route)
                    asgi_app.add_api_route(route.path, bound, methods=list(route.methods),
                                           response_model=route.response_model,
                                           status_code=route.status_code)

        cls.__serve_bind_asgi__ = __serve_bind_asgi__
        cls._serve_asgi_app = app
        cls.__init__ = orig_init
        return cls

    return deco


def _build(app: Application, app_name, specs: dict):
    dep = app.deployment
    if dep.name in specs:
        return DeploymentHandle(dep.name, app_name)

    def conv(v):
        if isinstance(v, Application):
            return _build(v, app_name, specs)
        if isinstance(v, (list, tuple)):
            return type(v)(conv(x) for x in v)
        if isinstance(v, dict):
            return {k: conv(x) for k, x in v.items()}
        return v

    args = tuple(conv(a) for a in app.args)
    kwargs = {k: conv(v) for k, v in app.kwargs.items()}
    fc = dep.func_or_class
    blob = cloudpickle.dumps(fc)
    asgi = getattr(fc, "_serve_asgi_app", None) if inspect.isclass(fc) else None
    specs[dep.name] = {
        "name": dep.name, "callable": blob, "is_function": not inspect.isclass(fc),
        "init_args": args, "init_kwargs": kwargs, "num_replicas": dep.num_replicas,
        "autoscaling_config": dep.autoscaling_config, "ray_actor_options": dep.ray_actor_options,
        "user_config": dep.user_config, "max_ongoing_requests": dep.max_ongoing_requests,
        "max_queued_requests": dep.max_queued_requests,
        "asgi_app": cloudpickle.dumps(asgi) if asgi is not None else None,
        "graceful_shutdown_timeout_s": dep.graceful_shutdown_timeout_s,
        "graceful_shutdown_wait_loop_s": dep.graceful_shutdown_wait_loop_s,
        "logging_config": dep.logging_config,
        "health_check_period_s": dep.health_check_period_s,
        "health_check_timeout_s": dep.health_check_timeout_s,
        "placement_group_bundles": dep.placement_group_bundles,
        "placement_group_strategy": dep.placement_group_strategy,
        "max_replicas_per_node": dep.max_replicas_per_node,
        "code_version": dep.version or hashlib.blake2b(blob, digest_size=8).hexdigest(),
    }
    return DeploymentHandle(dep.name, app_name)


def run(target: Application, *, name: str = "default", route_prefix: str | None = "/",
        blocking: bool = False, _blocking=None, **kw) -> DeploymentHandle:
    if isinstance(target, Deployment):
        target = target.bind()
    c = start(kw.get("http_options"), grpc_options=kw.get("grpc_options"))
    specs: dict = {}
    handle = _build(target, name, specs)
    rp = target.deployment.route_prefix or route_prefix
    ray.get(c.deploy_application.remote(name, rp, target.deployment.name, list(specs.values())))
    from ray_amd.serve import handle as H

    H.invalidate(name, drop=False)  # this process's routers re-read the new replica sets
    st = ray.get(c.status.remote()).get(name, {})
    if st.get("status") == "DEPLOY_FAILED":
        errs = {d: s["status"] for d, s in st.get("deployments", {}).items()}
        raise RuntimeError(f"application {name} failed to deploy: {errs}")
    if blocking:
        while True:
            time.sleep(1)
    return handle


_run = run  # reference: serve._run (internal alias used by tooling)


def delete(name: str, _blocking: bool = True):
    ray.get(_get_controller().delete_application.remote(name))
    from ray_amd.serve import handle as H

    H.invalidate(name)


def shutdown():
    global _controller, _proxy
    try:
        c = _get_controller()
    except Exception:
        return
    try:
        ray.get(c.shutdown.remote())
    except Exception:
        pass
    try:
        ray.kill(c)
    except Exception:
        pass
    _controller = None
    _proxy = None
    from ray_amd.serve import handle as H

    H._routers.clear()


def status():
    return ray.get(_get_controller().status.remote())


def get_app_handle(name: str) -> DeploymentHandle:
    ing = ray.get(_get_controller().get_ingress.remote(name))
    if ing is None:
        raise RuntimeError(f"application {name} does not exist")
    return DeploymentHandle(ing, name)


def get_deployment_handle(deployment_name: str, app_name: str = "default"):
    return DeploymentHandle(deployment_name, app_name)


def get_replica_context():
    from ray_amd.serve import context

    return context.get_replica_context()


def multiplexed(_fn=None, *, max_num_models_per_replica: int = 3):
    """Cache up to N loaded models per replica keyed by the request's multiplexed model id."""
    import collections
    import functools

    def deco(fn):
        cache = collections.OrderedDict()

        @functools.wraps(fn)
        async def wrapper(*args):
            model_id = args[-1]
            if model_id in cache:
                cache.move_to_end(model_id)
                return cache[model_id]
            r = fn(*args)
            if inspect.isawaitable(r):
                r = await r
            cache[model_id] = r
            while len(cache) > max_num_models_per_replica:
                cache.popitem(last=False)
            return r

        return wrapper

    if _fn is not None and callable(_fn):
        return deco(_fn)
    return deco


def get_multiplexed_model_id() -> str:
    from ray_amd.serve import context

    return context.current_model_id()
