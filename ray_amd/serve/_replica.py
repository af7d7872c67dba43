"""Serve replica actor (reference: python/ray/serve/_private/replica.py).

An async actor wrapping the user's deployment class/function. Tracks ongoing
requests (for power-of-two-choices routing and autoscaling), supports
``reconfigure(user_config)``, health checks, ASGI ingress (FastAPI/starlette
apps via ``@serve.ingress``) and plain ``__call__(request)`` HTTP handlers."""

from __future__ import annotations

import asyncio
import inspect
import time


class _Request:
    """Minimal starlette-compatible request built from the proxy's forwarded scope."""

    def __init__(self, scope, body: bytes):
        self.scope = scope
        self._body = body
        self.method = scope.get("method", "GET")
        self.url_path = scope.get("path", "/")
        self.headers = {k.decode() if isinstance(k, bytes) else k:
                        v.decode() if isinstance(v, bytes) else v
                        for k, v in scope.get("headers", [])}
        from urllib.parse import parse_qsl

        qs = scope.get("query_string", b"")
        self.query_params = dict(parse_qsl(qs.decode() if isinstance(qs, bytes) else qs))
        self.path_params = {}

    async def body(self):
        return self._body

    async def json(self):
        import json

        return json.loads(self._body or b"null")


async def _call_asgi(app, scope, body):
    sent = {"status": 500, "headers": [], "body": b""}
    chunks = [body]

    async def receive():
        if chunks:
            return {"type": "http.request", "body": chunks.pop(), "more_body": False}
        await asyncio.sleep(3600)
        return {"type": "http.disconnect"}

    async def send(msg):
        if msg["type"] == "http.response.start":
            sent["status"] = msg["status"]
            sent["headers"] = [(k.decode(), v.decode()) for k, v in msg.get("headers", [])]
        elif msg["type"] == "http.response.body":
            sent["body"] += msg.get("body", b"")

    s = dict(scope)
    s.setdefault("type", "http")
    s.setdefault("asgi", {"version": "3.0"})
    s.setdefault("http_version", "1.1")
    s.setdefault("scheme", "http")
    s.setdefault("server", ("127.0.0.1", 8000))
    s.setdefault("client", ("127.0.0.1", 0))
    s.setdefault("root_path", "")
    s["headers"] = [(k.encode() if isinstance(k, str) else k, v.encode() if isinstance(v, str)
                     else v) for k, v in s.get("headers", [])]
    await app(s, receive, send)
    return sent["status"], sent["headers"], sent["body"]


def _chunk_bytes(c):
    if isinstance(c, bytes):
        return c
    if isinstance(c, str):
        return c.encode()
    import json

    return json.dumps(c).encode()


def _streaming_body(result):
    """(status, headers, async iterator of bytes) for streamed results, else None."""
    try:
        from starlette.responses import StreamingResponse

        if isinstance(result, StreamingResponse):
            async def it():
                async for c in result.body_iterator:
                    yield _chunk_bytes(c)

            return (result.status_code, [(k, v) for k, v in result.headers.items()], it())
    except ImportError:
        pass
    if inspect.isasyncgen(result):
        async def ait():
            async for c in result:
                yield _chunk_bytes(c)

        return 200, [("content-type", "text/plain; charset=utf-8")], ait()
    if inspect.isgenerator(result):
        async def git():
            for c in result:
                yield _chunk_bytes(c)

        return 200, [("content-type", "text/plain; charset=utf-8")], git()
    return None


async def _stream_asgi(app, scope, body):
    """Run an ASGI app, yielding response messages as it sends them."""
    q: asyncio.Queue = asyncio.Queue()
    chunks = [body]

    async def receive():
        if chunks:
            return {"type": "http.request", "body": chunks.pop(), "more_body": False}
        await asyncio.sleep(3600)
        return {"type": "http.disconnect"}

    async def send(msg):
        await q.put(msg)

    s = dict(scope)
    s.setdefault("type", "http")
    s.setdefault("asgi", {"version": "3.0"})
    s.setdefault("http_version", "1.1")
    s.setdefault("scheme", "http")
    s.setdefault("server", ("127.0.0.1", 8000))
    s.setdefault("client", ("127.0.0.1", 0))
    s.setdefault("root_path", "")
    s["headers"] = [(k.encode() if isinstance(k, str) else k, v.encode() if isinstance(v, str)
                     else v) for k, v in s.get("headers", [])]
    task = asyncio.ensure_future(app(s, receive, send))
    done_sentinel = object()
    task.add_done_callback(lambda t: q.put_nowait(done_sentinel))
    while True:
        msg = await q.get()
        if msg is done_sentinel:
            break
        if msg["type"] == "http.response.start":
            yield ("start", msg["status"],
                   [(k.decode(), v.decode()) for k, v in msg.get("headers", [])])
        elif msg["type"] == "http.response.body":
            b = msg.get("body", b"")
            if b:
                yield ("body", b)
            if not msg.get("more_body"):
                break
    if task.done() and task.exception() is not None:
        raise task.exception()


def _to_http_response(result):
    import json

    try:
        from starlette.responses import Response

        if isinstance(result, Response):
            return result.status_code, [(k, v) for k, v in result.headers.items()], result.body
    except ImportError:
        pass
    if isinstance(result, bytes):
        return 200, [("content-type", "application/octet-stream")], result
    if isinstance(result, str):
        return 200, [("content-type", "text/plain; charset=utf-8")], result.encode()
    return 200, [("content-type", "application/json")], json.dumps(result).encode()


async def _resolve_args(args, kwargs):
    """DeploymentResponses passed as arguments arrive as ObjectRefs inside the request's
    args/kwargs: resolve them to values before the user method runs (reference: the
    router resolves DeploymentResponse arguments before assignment)."""
    from ray_amd.object_ref import ObjectRef

    if not any(isinstance(a, ObjectRef) for a in args) and \
            not any(isinstance(v, ObjectRef) for v in kwargs.values()):
        return args, kwargs
    args = [await a if isinstance(a, ObjectRef) else a for a in args]
    kwargs = {k: (await v if isinstance(v, ObjectRef) else v) for k, v in kwargs.items()}
    return tuple(args), kwargs


class Replica:
    def __init__(self, deployment_name, app_name, callable_blob, init_args, init_kwargs,
                 user_config, replica_id, is_function, asgi_app_blob):
        import cloudpickle

        self.deployment_name = deployment_name
        self.app_name = app_name
        self.replica_id = replica_id
        from ray_amd.serve import context as _ctx

        rc = _ctx.ReplicaContext(app_name, deployment_name, replica_id)
        _ctx._set_replica_context(rc)  # visible to the user's constructor too
        target = cloudpickle.loads(callable_blob)
        self.is_function = is_function
        if is_function:
            self.obj = target
        else:
            self.obj = target(*init_args, **init_kwargs)
        rc.servable_object = self.obj
        self.asgi = None
        if asgi_app_blob is not None:
            app = cloudpickle.loads(asgi_app_blob)
            self.asgi = app
            if hasattr(self.obj, "__serve_bind_asgi__"):
                self.obj.__serve_bind_asgi__(app)
        elif getattr(self.obj, "_serve_asgi_instance_app", None) is not None:
            # an ASGI app the constructor builds (gradio_integrations.GradioIngress)
            self.asgi = self.obj._serve_asgi_instance_app
        self.ongoing = 0
        self.total = 0
        self.started = time.time()
        self.user_config = None
        if user_config is not None:
            self._reconfigure(user_config)

    def _reconfigure(self, cfg):
        self.user_config = cfg
        f = getattr(self.obj, "reconfigure", None)
        if f is not None:
            r = f(cfg)
            if inspect.isawaitable(r):
                return r
        return None

    async def reconfigure(self, cfg):
        r = self._reconfigure(cfg)
        if r is not None:
            await r
        return True

    async def check_health(self):
        f = getattr(self.obj, "check_health", None)
        if f is not None:
            r = f()
            if inspect.isawaitable(r):
                await r
        return True

    def num_ongoing(self):
        return self.ongoing

    def stats(self):
        return {"ongoing": self.ongoing, "total": self.total, "replica_id": self.replica_id}

    async def handle_request(self, method_name, args, kwargs, multiplexed_model_id=""):
        from ray_amd.serve import context

        self.ongoing += 1
        self.total += 1
        token = context._set_request_context(multiplexed_model_id)
        t0 = time.perf_counter() if getattr(self, "access_log", False) else None
        status = "OK"
        try:
            args, kwargs = await _resolve_args(args, kwargs)
            if self.is_function:
                fn = self.obj
            else:
                fn = getattr(self.obj, method_name or "__call__")
            r = fn(*args, **kwargs)
            if inspect.isawaitable(r):
                r = await r
            if inspect.isgenerator(r):
                r = list(r)
            elif inspect.isasyncgen(r):
                r = [x async for x in r]
            return r
        except BaseException:
            status = "ERROR"
            raise
        finally:
            context._reset_request_context(token)
            self.ongoing -= 1
            if t0 is not None:  # logging_config enable_access_log: one line per request
                import logging

                logging.getLogger("ray.serve").info(
                    "%s %s %s %.1fms", self.deployment_name, method_name or "__call__",
                    status, (time.perf_counter() - t0) * 1e3)

    async def handle_http(self, scope, body):
        self.ongoing += 1
        self.total += 1
        try:
            if self.asgi is not None:
                return await _call_asgi(self.asgi, scope, body)
            req = _Request(scope, body)
            fn = self.obj if self.is_function else getattr(self.obj, "__call__")
            r = fn(req)
            if inspect.isawaitable(r):
                r = await r
            return _to_http_response(r)
        finally:
            self.ongoing -= 1

    async def handle_request_streaming(self, method_name, args, kwargs, multiplexed_model_id=""):
        """Streaming variant (handle.options(stream=True)): yields each item the user's
        generator / async generator produces as its own stream element."""
        from ray_amd.serve import context

        self.ongoing += 1
        self.total += 1
        token = context._set_request_context(multiplexed_model_id)
        try:
            args, kwargs = await _resolve_args(args, kwargs)
            fn = self.obj if self.is_function else getattr(self.obj, method_name or "__call__")
            r = fn(*args, **kwargs)
            if inspect.isawaitable(r):
                r = await r
            if inspect.isasyncgen(r):
                async for x in r:
                    yield x
            elif inspect.isgenerator(r):
                for x in r:
                    yield x
            else:
                yield r
        finally:
            context._reset_request_context(token)
            self.ongoing -= 1

    async def handle_http_streaming(self, scope, body):
        """HTTP with streamed responses: yields ("start", status, headers) then
        ("body", chunk) messages as the application produces them (ASGI apps: every
        ``http.response.body`` send; StreamingResponse / generator results: every chunk)."""
        self.ongoing += 1
        self.total += 1
        try:
            if self.asgi is not None:
                async for m in _stream_asgi(self.asgi, scope, body):
                    yield m
                return
            req = _Request(scope, body)
            fn = self.obj if self.is_function else getattr(self.obj, "__call__")
            r = fn(req)
            if inspect.isawaitable(r):
                r = await r
            it = _streaming_body(r)
            if it is not None:
                status, headers, chunks = it
                yield ("start", status, headers)
                async for c in chunks:
                    yield ("body", c)
                return
            status, headers, out = _to_http_response(r)
            yield ("start", status, headers)
            yield ("body", out)
        finally:
            self.ongoing -= 1

    def set_logging(self, cfg: dict):
        """Deployment logging_config: the replica's Python log level (root and the user
        code's loggers) and whether it logs one access line per request."""
        import logging

        logging.getLogger().setLevel(cfg.get("log_level", "INFO"))
        self.access_log = bool(cfg.get("enable_access_log", True))
        return True

    async def prepare_for_shutdown(self, wait_loop_s: float = 2.0):
        """Wait until no request is in flight, checking every ``wait_loop_s`` seconds
        (graceful_shutdown_wait_loop_s); the controller bounds the whole wait by
        graceful_shutdown_timeout_s."""
        self.draining = True
        while self.ongoing > 0:
            await asyncio.sleep(wait_loop_s)
        f = getattr(self.obj, "__del__", None)
        return True
