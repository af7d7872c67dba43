"""HTTP proxy actor (reference: python/ray/serve/_private/proxy.py, proxy_router.py).

Runs uvicorn + a raw ASGI app in a background thread inside an actor; each
request is matched by longest route prefix and forwarded to the ingress
deployment's replica (``handle_http``) chosen by the handle router."""

from __future__ import annotations

import asyncio
import threading
import time


class HTTPProxy:
    def __init__(self, host="127.0.0.1", port=8000):
        self.host = host
        self.port = port
        self.routes = {}
        self.routes_ts = 0.0
        self.ready = threading.Event()
        self.error = None
        t = threading.Thread(target=self._serve, daemon=True)
        t.start()
        self.ready.wait(30)

    def _refresh(self):
        if time.time() - self.routes_ts > 0.5:
            import ray_amd as ray
            from ray_amd.serve.api import _get_controller

            self.routes = ray.get(_get_controller().get_routes.remote())
            self.routes_ts = time.time()

    def _match(self, path):
        best = None
        for prefix, target in self.routes.items():
            p = prefix.rstrip("/") or "/"
            if path == p or path.startswith(p.rstrip("/") + "/") or p == "/":
                if best is None or len(p) > len(best[0]):
                    best = (p, target)
        return best

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
        loop = asyncio.get_running_loop()
        try:
            await loop.run_in_executor(None, self._refresh)
            hit = self._match(scope["path"])
            if hit is None:
                status, headers, out = 404, [("content-type", "text/plain")], \
                    f"Path '{scope['path']}' not found".encode()
            else:
                prefix, (app_name, ingress) = hit
                fwd = {k: v for k, v in scope.items() if k in ("method", "path", "query_string",
                                                               "headers", "type",
                                                               "http_version", "scheme")}
                fwd["headers"] = [(k.decode(), v.decode()) for k, v in scope.get("headers", [])]
                if prefix != "/":
                    fwd["root_path"] = ""
                    fwd["path"] = scope["path"][len(prefix):] or "/"
                status, headers, out = await loop.run_in_executor(
                    None, self._forward, app_name, ingress, fwd, body)
        except Exception as e:  # noqa: BLE001
            status, headers, out = 500, [("content-type", "text/plain")], repr(e).encode()
        await send({"type": "http.response.start", "status": status,
                    "headers": [(k.encode(), v.encode()) for k, v in headers]})
        await send({"type": "http.response.body", "body": out})

    def _forward(self, app_name, ingress, scope, body):
        import ray_amd as ray
        from ray_amd.serve.handle import _router

        r = _router(app_name, ingress)
        rid, h = r.choose()
        try:
            return ray.get(h.handle_http.remote(scope, body))
        finally:
            r.done(rid)

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
