"""HTTP proxy actor (reference: python/ray/serve/_private/proxy.py, proxy_router.py;
``send_request_to_replica`` streaming path, proxy.py:518).

Runs uvicorn + a raw ASGI app on its own event loop inside an actor; each request is
matched by longest route prefix and forwarded to the ingress deployment's replica
chosen by the handle router. Forwarding is fully asynchronous: the route table and
replica set are refreshed with awaited controller calls, and the response comes back
as a streaming generator (``handle_http_streaming``) whose messages are written to the
client as they arrive (chunked transfer for streamed bodies) — no blocking ``ray.get``
and no thread per request."""

from __future__ import annotations

import asyncio
import threading
import time


class HTTPProxy:
    def __init__(self, host="127.0.0.1", port=8000, request_timeout_s=None):
        self.host = host
        self.port = port
        # HTTPOptions.request_timeout_s: a request not answered by then gets 408 (reference
        # proxy.py request_timeout_s -> "Request timed out", status 408)
        self.request_timeout_s = request_timeout_s if request_timeout_s and \
            request_timeout_s > 0 else None
        self.num_timeouts = 0
        self.routes = {}
        self.routes_ts = 0.0
        self.inflight = 0
        self.ready = threading.Event()
        self.error = None
        t = threading.Thread(target=self._serve, daemon=True)
        t.start()
        self.ready.wait(30)

    def _match(self, path):
        best = None
        for prefix, target in self.routes.items():
            p = prefix.rstrip("/") or "/"
            if path == p or path.startswith(p.rstrip("/") + "/") or p == "/":
                if best is None or len(p) > len(best[0]):
                    best = (p, target)
        return best

    async def _arefresh(self):
        if time.time() - self.routes_ts > 0.5:
            from ray_amd.serve.api import _get_controller

            self.routes = await _get_controller().get_routes.remote()
            self.routes_ts = time.time()

    async def _app(self, scope, receive, send):
        if scope["type"] == "lifespan":
            while True:
                m = await receive()
                if m["type"] == "lifespan.startup":
                    await send({"type": "lifespan.startup.complete"})
                elif m["type"] == "lifespan.shutdown":
                    await send({"type": "lifespan.shutdown.complete"})
                    return
        if scope["type"] != "http":
            return
        body = b""
        while True:
            m = await receive()
            body += m.get("body", b"")
            if not m.get("more_body"):
                break
        state = {"started": False}
        if self.request_timeout_s is None:
            await self._handle(scope, body, send, state)
            return
        try:
            await asyncio.wait_for(self._handle(scope, body, send, state),
                                   self.request_timeout_s)
        except asyncio.TimeoutError:
            self.num_timeouts += 1
            if not state["started"]:
                await self._reply(send, 408, [("content-type", "text/plain")],
                                  f"Request timed out after {self.request_timeout_s}s."
                                  .encode())

    async def _handle(self, scope, body, send, state):
        started = False
        try:
            await self._arefresh()
            hit = self._match(scope["path"])
            if hit is None:  # a route deployed since the last refresh: look again once
                self.routes_ts = 0.0
                await self._arefresh()
                hit = self._match(scope["path"])
            if hit is None:
                await self._reply(send, 404, [("content-type", "text/plain")],
                                  f"Path '{scope['path']}' not found".encode())
                return
            prefix, (app_name, ingress) = hit
            fwd = {k: v for k, v in scope.items() if k in ("method", "path", "query_string",
                                                           "headers", "type", "http_version",
                                                           "scheme")}
            fwd["headers"] = [(k.decode(), v.decode()) for k, v in scope.get("headers", [])]
            if prefix != "/":
                fwd["root_path"] = ""
                fwd["path"] = scope["path"][len(prefix):] or "/"
            from ray_amd.serve.exceptions import BackPressureError
            from ray_amd.serve.handle import _is_replica_death, _router

            r = _router(app_name, ingress)
            for attempt in range(2):
                try:
                    rid, h = await r.achoose()
                except BackPressureError as e:
                    await self._reply(send, 503, [("content-type", "text/plain")],
                                      e.message.encode())
                    return
                except RuntimeError:  # the app was deleted since the routes were read
                    self.routes_ts = 0.0
                    await self._arefresh()
                    if self._match(scope["path"]) is None:
                        await self._reply(send, 404, [("content-type", "text/plain")],
                                          f"Path '{scope['path']}' not found".encode())
                        return
                    raise
                self.inflight += 1
                try:
                    gen = h.handle_http_streaming.remote(fwd, body)
                    async for ref in gen:
                        msg = await ref
                        if msg[0] == "start":
                            await send({"type": "http.response.start", "status": msg[1],
                                        "headers": [(k.encode(), v.encode())
                                                    for k, v in msg[2]]})
                            started = state["started"] = True
                        else:
                            await send({"type": "http.response.body", "body": msg[1],
                                        "more_body": True})
                    if not started:
                        raise RuntimeError("replica produced no response")
                    await send({"type": "http.response.body", "body": b"",
                                "more_body": False})
                    return
                except Exception as e:  # noqa: BLE001
                    # the replica died before answering (redeploy / scale-down raced the
                    # cached routing table): once more on a freshly read replica set
                    if started or attempt or not _is_replica_death(e):
                        raise
                    await r.arefresh(force=True)
                finally:
                    self.inflight -= 1
                    r.done(rid)
        except Exception as e:  # noqa: BLE001
            if not started:
                await self._reply(send, 500, [("content-type", "text/plain")], repr(e).encode())

    def invalidate_routes(self, app_name=None):
        """Pushed by the controller after a deploy or delete."""
        self.routes_ts = 0.0
        if app_name is not None:
            from ray_amd.serve.handle import invalidate

            invalidate(app_name, drop=False)
        return True

    @staticmethod
    async def _reply(send, status, headers, out):
        await send({"type": "http.response.start", "status": status,
                    "headers": [(k.encode(), v.encode()) for k, v in headers]})
        await send({"type": "http.response.body", "body": out})

    def num_inflight(self):
        return self.inflight

    def stats(self):
        return {"inflight": self.inflight, "timeouts": self.num_timeouts}

    def _serve(self):
        try:
            import uvicorn

            cfg = uvicorn.Config(self._app, host=self.host, port=self.port, log_level="error",
                                 lifespan="on", interface="asgi3")
            server = uvicorn.Server(cfg)
            loop = asyncio.new_event_loop()
            asyncio.set_event_loop(loop)

            async def watch():
                while not server.started:
                    await asyncio.sleep(0.01)
                self.ready.set()

            async def run():
                loop.create_task(watch())
                await server.serve()

            loop.run_until_complete(run())
        except Exception as e:  # noqa: BLE001
            self.error = repr(e)
            self.ready.set()

    def ping(self):
        return self.error or "ok"
