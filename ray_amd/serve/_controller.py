"""Serve controller (reference: python/ray/serve/_private/{controller,deployment_state,
application_state,autoscaling_policy}.py).

A detached async actor that owns the applications → deployments → replica
actors mapping, reconciles replica counts, runs the autoscaling policy
(target ongoing requests per replica, bounded by min/max replicas, with up/down
smoothing delays) and serves routing tables to handles and the HTTP proxy."""

from __future__ import annotations

import asyncio
import math
import time
import uuid

import ray_amd as ray

CONTROLLER_NAME = "SERVE_CONTROLLER_ACTOR"
SERVE_NAMESPACE = "serve"


class _DeploymentState:
    def __init__(self, app, spec):
        self.app = app
        self.spec = spec
        self.name = spec["name"]
        self.replicas = {}  # replica_id -> handle
        self.version = 0
        self.target = spec["num_replicas"]
        asc = spec.get("autoscaling_config")
        if asc:
            self.target = asc.get("initial_replicas") or asc.get("min_replicas", 1)
        self.last_scale = time.time()
        self.status = "UPDATING"
        self.over_since = None
        self.under_since = None
        self.retiring = {}  # old-version replicas serving until their successors are up


class ServeController:
    def __init__(self, http_options=None):
        self.apps = {}  # app name -> {"route_prefix", "ingress", "deployments": {name: state}}
        self.http_options = http_options or {}
        self.proxy = None
        self._loop_task = None

    async def _ensure_loop(self):
        if self._loop_task is None:
            self._loop_task = asyncio.get_running_loop().create_task(self._control_loop())

    async def deploy_application(self, app_name, route_prefix, ingress, deployments):
        await self._ensure_loop()
        old = self.apps.get(app_name)
        states = {}
        for spec in deployments:
            st = None
            if old and spec["name"] in old["deployments"]:
                st = old["deployments"][spec["name"]]
                code_changed = st.spec.get("code_version") != spec.get("code_version")
                cfg_changed = st.spec.get("user_config") != spec.get("user_config")
                st.spec = spec
                if not spec.get("autoscaling_config"):
                    st.target = spec["num_replicas"]
                if code_changed:
                    # rolling update: the old replicas keep serving until the new ones
                    # pass their health check, then drain (reference:
                    # deployment_state.py version-mismatched replicas)
                    st.retiring = dict(st.replicas)
                    st.replicas = {}
                elif cfg_changed and spec.get("user_config") is not None:
                    await asyncio.gather(*[r.reconfigure.remote(spec["user_config"])
                                           for r in st.replicas.values()])
            else:
                st = _DeploymentState(app_name, spec)
            states[spec["name"]] = st
        if old:
            for name, st in old["deployments"].items():
                if name not in states:
                    await self._stop_replicas(st, list(st.replicas))
        self.apps[app_name] = {"route_prefix": route_prefix, "ingress": ingress,
                               "deployments": states, "status": "DEPLOYING"}
        await self._reconcile()
        await self._push_routes(app_name)
        return True

    async def _push_routes(self, app_name):
        if self.proxy is not None:
            try:
                await self.proxy.invalidate_routes.remote(app_name)
            except Exception:  # noqa: BLE001
                pass

    async def _start_replica(self, st):
        spec = st.spec
        from ray_amd.serve._replica import Replica

        rid = f"{st.name}#{uuid.uuid4().hex[:6]}"
        opts = dict(spec.get("ray_actor_options") or {})
        opts.setdefault("num_cpus", 0)
        opts["max_concurrency"] = max(100, spec.get("max_ongoing_requests", 100) * 2)
        cls = ray.remote(Replica)
        h = cls.options(**opts).remote(st.name, st.app, spec["callable"], spec["init_args"],
                                       spec["init_kwargs"], spec.get("user_config"), rid,
                                       spec["is_function"], spec.get("asgi_app"))
        st.replicas[rid] = h
        return rid, h

    async def _drain(self, st, replicas):
        """Stop replicas that are no longer routed to, after their in-flight requests."""
        saved = st.replicas
        st.replicas = dict(replicas)
        try:
            await self._stop_replicas(st, list(replicas))
        finally:
            st.replicas = saved

    async def _stop_replicas(self, st, rids):
        for rid in rids:
            h = st.replicas.pop(rid, None)
            if h is not None:
                try:
                    await asyncio.wait_for(h.prepare_for_shutdown.remote(),
                                           st.spec.get("graceful_shutdown_timeout_s", 5))
                except Exception:
                    pass
                ray.kill(h)
        st.version += 1

    async def _reconcile(self):
        for app in list(self.apps.values()):
            all_ok = True
            for st in list(app["deployments"].values()):
                diff = st.target - len(st.replicas)
                if diff > 0:
                    started = [await self._start_replica(st) for _ in range(diff)]
                    # wait for constructors
                    try:
                        await asyncio.gather(*[h.check_health.remote() for _, h in started])
                        st.status = "HEALTHY"
                    except Exception as e:  # noqa: BLE001
                        st.status = "UNHEALTHY"
                        st.error = repr(e)
                        for rid, _ in started:
                            st.replicas.pop(rid, None)
                        all_ok = False
                    st.version += 1
                    if st.retiring and st.status == "HEALTHY":
                        old, st.retiring = st.retiring, {}
                        await self._drain(st, old)
                elif diff < 0:
                    await self._stop_replicas(st, list(st.replicas)[:(-diff)])
                    st.status = "HEALTHY"
                else:
                    st.status = "HEALTHY" if st.status != "UNHEALTHY" else st.status
                all_ok = all_ok and st.status == "HEALTHY"
            app["status"] = "RUNNING" if all_ok else "DEPLOY_FAILED"

    async def _autoscale(self):
        now = time.time()
        for app in list(self.apps.values()):
            for st in list(app["deployments"].values()):
                asc = st.spec.get("autoscaling_config")
                if not asc or not st.replicas:
                    continue
                try:
                    ongoing = await asyncio.gather(*[h.num_ongoing.remote()
                                                     for h in st.replicas.values()])
                except Exception:
                    continue
                total = sum(ongoing)
                tgt = asc.get("target_ongoing_requests", asc.get(
                    "target_num_ongoing_requests_per_replica", 2))
                desired = math.ceil(total / max(tgt, 1e-9)) if total else \
                    asc.get("min_replicas", 1)
                cur = len(st.replicas)
                # gain on each decision (reference: AutoscalingConfig.upscaling_factor /
                # downscaling_factor): move only that fraction of the way to the target
                if desired > cur and asc.get("upscaling_factor"):
                    desired = cur + math.ceil((desired - cur) * asc["upscaling_factor"])
                elif desired < cur and asc.get("downscaling_factor"):
                    desired = cur - max(1, math.floor((cur - desired) *
                                                      asc["downscaling_factor"]))
                desired = max(asc.get("min_replicas", 1), min(asc.get("max_replicas", 10),
                                                              desired))
                if desired > cur:
                    st.under_since = None
                    st.over_since = st.over_since or now
                    if now - st.over_since >= asc.get("upscale_delay_s", 0.5):
                        st.target = desired
                        st.over_since = None
                elif desired < cur:
                    st.over_since = None
                    st.under_since = st.under_since or now
                    if now - st.under_since >= asc.get("downscale_delay_s", 5.0):
                        st.target = desired
                        st.under_since = None
                else:
                    st.over_since = st.under_since = None

    async def _control_loop(self):
        while True:
            try:
                await self._autoscale()
                await self._reconcile()
                await self._health_check()
            except Exception:
                import traceback

                traceback.print_exc()
            await asyncio.sleep(0.2)

    async def _health_check(self):
        for app in list(self.apps.values()):
            for st in list(app["deployments"].values()):
                dead = []
                for rid, h in list(st.replicas.items()):
                    try:
                        await asyncio.wait_for(h.check_health.remote(), 10)
                    except Exception:
                        dead.append(rid)
                for rid in dead:
                    st.replicas.pop(rid, None)
                    st.version += 1

    def get_replicas(self, app_name, deployment_name):
        app = self.apps.get(app_name)
        if app is None or deployment_name not in app["deployments"]:
            return None
        st = app["deployments"][deployment_name]
        # during a rolling update the old version serves until the new one is up
        reps = st.replicas if st.replicas or not st.retiring else st.retiring
        return (st.version, list(reps.items()), st.spec.get("max_ongoing_requests", 100),
                st.spec.get("max_queued_requests", -1))

    def get_routes(self):
        return {a["route_prefix"]: (name, a["ingress"]) for name, a in self.apps.items()
                if a["route_prefix"] is not None}

    def get_ingress(self, app_name):
        a = self.apps.get(app_name)
        return None if a is None else a["ingress"]

    async def delete_application(self, app_name):
        app = self.apps.pop(app_name, None)
        if app:
            for st in list(app["deployments"].values()):
                if st.retiring:
                    old, st.retiring = st.retiring, {}
                    await self._drain(st, old)
                await self._stop_replicas(st, list(st.replicas))
            await self._push_routes(app_name)
        return True

    def status(self):
        out = {}
        for name, a in self.apps.items():
            out[name] = {"status": a["status"], "route_prefix": a["route_prefix"],
                         "deployments": {d: {"status": st.status, "replica_states":
                                             {"RUNNING": len(st.replicas)},
                                             "target_num_replicas": st.target}
                                         for d, st in a["deployments"].items()}}
        return out

    async def shutdown(self):
        for name in list(self.apps):
            await self.delete_application(name)
        for p in (self.proxy, getattr(self, "grpc_proxy", None)):
            if p is not None:
                try:
                    ray.kill(p)
                except Exception:
                    pass
        return True

    def set_proxy(self, proxy):
        self.proxy = proxy
        return True

    def get_proxy(self):
        return self.proxy

    def set_grpc_proxy(self, proxy):
        self.grpc_proxy = proxy
        return True

    def get_grpc_proxy(self):
        return getattr(self, "grpc_proxy", None)
