"""HTTP head: state API, cluster status, Prometheus metrics and the job REST API.

Parity with the reference dashboard head's JSON routes
(``dashboard/state_aggregator.py`` → ``/api/v0/<resource>``, ``/api/v0/tasks/summarize``;
``dashboard/modules/job/job_head.py`` → ``/api/jobs/``; ``/api/cluster_status``;
``/metrics``). No web UI. Served by uvicorn/starlette in its own process, connected to
the cluster as a driver; blocking cluster queries run in the threadpool.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys

from starlette.applications import Starlette
from starlette.concurrency import run_in_threadpool
from starlette.requests import Request
from starlette.responses import JSONResponse, PlainTextResponse, StreamingResponse
from starlette.routing import Route

import ray_amd as ray
from ray_amd.dashboard.job_manager import JobManager, JobStatus
from ray_amd.util import state as st

_LISTS = {"actors": st.list_actors, "tasks": st.list_tasks, "objects": st.list_objects,
          "nodes": st.list_nodes, "workers": st.list_workers, "jobs": st.list_jobs,
          "placement_groups": st.list_placement_groups, "runtime_envs": st.list_runtime_envs}
_SUMMARIES = {"tasks": st.summarize_tasks, "actors": st.summarize_actors,
              "objects": st.summarize_objects}


def _ok(data, status=200):
    return JSONResponse({"result": True, "msg": "", "data": data}, status_code=status)


def build_app(manager: JobManager) -> Starlette:
    async def version(_req):
        return JSONResponse({"version": "ray_amd", "ray_version": ray.__version__,
                             "session_name": os.path.basename(manager.session_dir)})

    async def cluster_status(_req):
        tot = await run_in_threadpool(ray.cluster_resources)
        av = await run_in_threadpool(ray.available_resources)
        return _ok({"clusterStatus": {"totalResources": tot, "availableResources": av}})

    async def state_list(req: Request):
        res = req.path_params["resource"]
        fn = _LISTS.get(res)
        if fn is None:
            return JSONResponse({"result": False, "msg": f"unknown resource {res}"}, 404)
        q = req.query_params
        keys = q.getlist("filter_keys")
        preds = q.getlist("filter_predicates")
        vals = q.getlist("filter_values")
        filters = list(zip(keys, preds, vals))
        limit = int(q.get("limit", 100))
        rows = await run_in_threadpool(lambda: fn(filters=filters, limit=None))
        return _ok({"result": {"result": [dict(r) for r in rows[:limit]], "total": len(rows),
                               "num_after_truncation": min(limit, len(rows)),
                               "num_filtered": len(rows)}})

    async def state_summary(req: Request):
        fn = _SUMMARIES.get(req.path_params["resource"])
        if fn is None:
            return JSONResponse({"result": False, "msg": "unknown resource"}, 404)
        return _ok({"result": await run_in_threadpool(fn)})

    async def metrics(_req):
        from ray_amd.util.metrics import prometheus_text

        return PlainTextResponse(await run_in_threadpool(prometheus_text),
                                 media_type="text/plain; version=0.0.4")

    # ------------------------------------------------------------------ jobs
    async def submit(req: Request):
        body = await req.json()
        if "entrypoint" not in body:
            return JSONResponse({"error": "entrypoint is required"}, 400)
        kw = {k: body.get(k) for k in ("entrypoint", "runtime_env", "metadata",
                                       "entrypoint_num_cpus", "entrypoint_num_gpus",
                                       "entrypoint_memory", "entrypoint_resources")}
        kw["submission_id"] = body.get("submission_id") or body.get("job_id")
        try:
            jid = await run_in_threadpool(lambda: manager.submit_job(**kw))
        except ValueError as e:
            return JSONResponse({"error": str(e)}, 400)
        return JSONResponse({"submission_id": jid, "job_id": jid})

    async def list_jobs(_req):
        jobs = await run_in_threadpool(manager.list_jobs)
        return JSONResponse(list(jobs.values()))

    async def job_info(req: Request):
        info = await run_in_threadpool(manager.get_job_info, req.path_params["job_id"])
        if info is None:
            return JSONResponse({"error": "job not found"}, 404)
        return JSONResponse(info)

    async def job_logs(req: Request):
        jid = req.path_params["job_id"]
        if await run_in_threadpool(manager.get_job_info, jid) is None:
            return JSONResponse({"error": "job not found"}, 404)
        return JSONResponse({"logs": await run_in_threadpool(manager.get_job_logs, jid)})

    async def job_logs_tail(req: Request):
        jid = req.path_params["job_id"]

        async def gen():
            sent = 0
            while True:
                logs = await run_in_threadpool(manager.get_job_logs, jid)
                if len(logs) > sent:
                    yield logs[sent:]
                    sent = len(logs)
                info = await run_in_threadpool(manager.get_job_info, jid)
                if info is None or JobStatus(info["status"]).is_terminal():
                    logs = await run_in_threadpool(manager.get_job_logs, jid)
                    if len(logs) > sent:
                        yield logs[sent:]
                    return
                await asyncio.sleep(0.2)

        return StreamingResponse(gen(), media_type="text/plain")

    async def job_stop(req: Request):
        try:
            ok = await run_in_threadpool(manager.stop_job, req.path_params["job_id"])
        except ValueError as e:
            return JSONResponse({"error": str(e)}, 404)
        return JSONResponse({"stopped": ok})

    async def job_delete(req: Request):
        try:
            ok = await run_in_threadpool(manager.delete_job, req.path_params["job_id"])
        except ValueError as e:
            return JSONResponse({"error": str(e)}, 404)
        except RuntimeError as e:
            return JSONResponse({"error": str(e)}, 400)
        return JSONResponse({"deleted": ok})

    # ---- Serve REST API (reference: dashboard/modules/serve/serve_head.py)
    def _serve_details():
        from ray_amd import serve
        from ray_amd.serve.schema import get_deployed_config

        try:
            st_ = serve.status()
        except RuntimeError:
            st_ = {}
        cfg = get_deployed_config() or {}
        apps = {}
        for a in cfg.get("applications", []):
            if a.get("name") in st_:
                apps[a["name"]] = {"deployed_app_config": a}
        for name, info in st_.items():
            apps.setdefault(name, {})
            apps[name].update({"name": name, "status": info.get("status"),
                               "route_prefix": info.get("route_prefix"),
                               "deployments": info.get("deployments", {})})
        return {"proxy_location": cfg.get("proxy_location", "EveryNode"),
                "http_options": cfg.get("http_options"), "applications": apps}

    async def serve_get(_req):
        return JSONResponse(await run_in_threadpool(_serve_details))

    async def serve_put(req: Request):
        from pydantic import ValidationError

        from ray_amd.serve.schema import ServeDeploySchema, deploy_config

        try:
            cfg = ServeDeploySchema(**(await req.json()))
        except (ValidationError, ValueError, TypeError) as e:
            return PlainTextResponse(str(e), 400)
        try:
            await run_in_threadpool(deploy_config, cfg)
        except Exception as e:  # noqa: BLE001
            return PlainTextResponse(f"deploy failed: {e!r}", 500)
        return PlainTextResponse("")

    async def serve_delete(_req):
        from ray_amd import serve

        await run_in_threadpool(serve.shutdown)
        return PlainTextResponse("")

    routes = [
        Route("/api/serve/applications/", serve_get, methods=["GET"]),
        Route("/api/serve/applications/", serve_put, methods=["PUT"]),
        Route("/api/serve/applications/", serve_delete, methods=["DELETE"]),
        Route("/api/version", version),
        Route("/api/cluster_status", cluster_status),
        Route("/api/v0/{resource}/summarize", state_summary),
        Route("/api/v0/{resource}", state_list),
        Route("/metrics", metrics),
        Route("/api/jobs/", submit, methods=["POST"]),
        Route("/api/jobs/", list_jobs, methods=["GET"]),
        Route("/api/jobs/{job_id}", job_info, methods=["GET"]),
        Route("/api/jobs/{job_id}", job_delete, methods=["DELETE"]),
        Route("/api/jobs/{job_id}/logs", job_logs),
        Route("/api/jobs/{job_id}/logs/tail", job_logs_tail),
        Route("/api/jobs/{job_id}/stop", job_stop, methods=["POST"]),
    ]
    return Starlette(routes=routes)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--session-dir", required=True)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8265)
    args = ap.parse_args(argv)
    import uvicorn

    ray.init(address=args.session_dir, namespace="_dashboard")
    manager = JobManager(args.session_dir)
    app = build_app(manager)
    config = uvicorn.Config(app, host=args.host, port=args.port, log_level="warning",
                            interface="asgi3")
    server = uvicorn.Server(config)
    url_file = os.path.join(args.session_dir, "dashboard.json")

    async def serve():
        task = asyncio.ensure_future(server.serve())
        while not server.started:
            if task.done():
                task.result()
                return
            await asyncio.sleep(0.02)
        with open(url_file + ".tmp", "w") as f:
            json.dump({"url": f"http://{args.host}:{args.port}", "pid": os.getpid()}, f)
        os.replace(url_file + ".tmp", url_file)
        await task

    asyncio.run(serve())
    sys.exit(0)


if __name__ == "__main__":
    main()
