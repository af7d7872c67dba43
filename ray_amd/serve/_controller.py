"""Serve controller (reference: python/ray/serve/_private/{controller,deployment_state,
application_state,autoscaling_policy,deployment_scheduler,long_poll}.py).

A detached, restartable async actor that owns the applications -> deployments -> replica
actors mapping. Its control loop never blocks on a replica:

* replica starts, health checks (every ``health_check_period_s``, failing after
  ``health_check_timeout_s``), load probes and drains all run as background tasks, so one
  slow or hung replica never stalls reconciliation or autoscaling of any application;
* autoscaling averages (ongoing requests at replicas + requests queued at handles, which
  handles push with ``record_handle_metrics``) over ``look_back_period_s``;
* replicas are placed by a deployment scheduler (spread over nodes, ``max_replicas_per_node``,
  one placement group per replica for ``placement_group_bundles``) and are named detached
  actors, so the controller checkpoints its state to the internal KV after every change and
  a restarted controller re-adopts the live replicas (reference controller.py:489, 524);
* handles and proxies receive replica-set changes by long poll (``long_poll``) instead of
  polling ``get_replicas``."""

from __future__ import annotations

import asyncio
import time
import uuid
from collections import deque

import ray_amd as ray
from ray_amd.serve.autoscaling_policy import resolve_policy

CONTROLLER_NAME = "SERVE_CONTROLLER_ACTOR"
SERVE_NAMESPACE = "serve"
CHECKPOINT_KEY = b"serve_controller_checkpoint"
KV_NAMESPACE = "serve"
TICK_S = 0.1
MAX_START_FAILURES = 3


def _replica_actor_name(app, rid):
    return f"SERVE_REPLICA::{app}::{rid}"


class _DeploymentState:
    def __init__(self, app, spec):
        self.app = app
        self.spec = spec
        self.name = spec["name"]
        self.replicas = {}  # replica_id -> handle (RUNNING: routed to)
        self.starting = {}  # replica_id -> handle (constructor / first health check pending)
        self.stopping = set()
        self.version = 0
        self.target = spec["num_replicas"]
        asc = spec.get("autoscaling_config")
        if asc:
            self.target = asc.get("initial_replicas") or asc.get("min_replicas", 1)
        self.status = "UPDATING"
        self.error = None
        self.start_failures = 0
        self.policy_state = {}  # the autoscaling policy's memory between ticks
        self.retiring = {}  # old-version replicas serving until their successors are up
        self.hc = {}  # rid -> (last check start time, task or None, consecutive failures)
        self.load = {}  # rid -> (ongoing, time)
        self.load_tasks = {}
        self.handle_queued = {}  # handle id -> (queued, time received)
        self.samples = deque()  # (time, total load)
        self.node_of = {}  # rid -> node id chosen by the scheduler
        self.pgs = {}  # rid -> placement group

    def period(self):
        return float(self.spec.get("health_check_period_s", 10.0))

    def hc_timeout(self):
        return float(self.spec.get("health_check_timeout_s", 30.0))


class _DeploymentScheduler:
    """Chooses where a new replica goes (reference: deployment_scheduler.py:245,592):
    a replica with ``placement_group_bundles`` gets its own placement group (the replica
    runs in bundle 0); otherwise replicas spread over the alive nodes that can hold one —
    fewest replicas of this deployment first, at most ``max_replicas_per_node`` — through a
    soft node-affinity strategy."""

    def actor_options(self, st, rid):
        from ray_amd.util.scheduling_strategies import (NodeAffinitySchedulingStrategy,
                                                        PlacementGroupSchedulingStrategy)

        spec = st.spec
        opts = dict(spec.get("ray_actor_options") or {})
        opts.setdefault("num_cpus", 0)
        bundles = spec.get("placement_group_bundles")
        if bundles:
            from ray_amd.util.placement_group import placement_group

            pg = placement_group(bundles, strategy=spec.get("placement_group_strategy") or
                                 "PACK")
            st.pgs[rid] = pg
            opts["scheduling_strategy"] = PlacementGroupSchedulingStrategy(
                pg, placement_group_bundle_index=0, placement_group_capture_child_tasks=True)
            return opts
        if "scheduling_strategy" in opts:
            return opts
        node = self._pick_node(st, opts)
        if node is not None:
            st.node_of[rid] = node
            opts["scheduling_strategy"] = NodeAffinitySchedulingStrategy(node, soft=True)
        return opts

    @staticmethod
    def _pick_node(st, opts):
        try:
            nodes = [n for n in ray.nodes() if n.get("Alive", n.get("alive", True))]
        except Exception:  # noqa: BLE001
            return None
        if len(nodes) <= 1:
            return None
        need = {"CPU": float(opts.get("num_cpus", 0) or 0),
                "GPU": float(opts.get("num_gpus", 0) or 0)}
        need.update({k: float(v) for k, v in (opts.get("resources") or {}).items()})
        per_node = {}
        for rid, node in st.node_of.items():
            if rid in st.replicas or rid in st.starting:
                per_node[node] = per_node.get(node, 0) + 1
        cap = st.spec.get("max_replicas_per_node")
        best, best_key = None, None
        for n in nodes:
            nid = n.get("NodeID") or n.get("node_id")
            total = n.get("Resources") or n.get("resources") or {}
            if any(total.get(k, 0.0) < v for k, v in need.items() if v):
                continue
            cnt = per_node.get(nid, 0)
            if cap and cnt >= cap:
                continue
            key = (cnt, -float(total.get("CPU", 0)))
            if best_key is None or key < best_key:
                best, best_key = nid, key
        return best


PROXY_TICK_S = 1.0  # per-node proxy reconciliation period (EveryNode)


class ServeController:
    def __init__(self, http_options=None):
        self.apps = {}  # app name -> {"route_prefix", "ingress", "deployments", "status"}
        self.http_options = http_options or {}
        self.proxy = None
        self.grpc_proxy = None
        self._loop_task = None
        self._changed = None  # asyncio.Event, replaced after each notification
        self._sched = _DeploymentScheduler()
        self._bg = set()
        self.recovered = False
        self._recovery = self._read_checkpoint()

    # ------------------------------------------------------------------ checkpoint
    @staticmethod
    def _read_checkpoint():
        try:
            from ray_amd.experimental import internal_kv

            blob = internal_kv._internal_kv_get(CHECKPOINT_KEY, namespace=KV_NAMESPACE)
        except Exception:  # noqa: BLE001
            return None
        if not blob:
            return None
        import cloudpickle

        try:
            return cloudpickle.loads(blob)
        except Exception:  # noqa: BLE001
            return None

    def _checkpoint(self):
        """Persist what a restarted controller needs: every app's specs and targets and
        the names of its replicas (reference controller.py:489 checkpoint to the KV)."""
        import cloudpickle

        state = {"http_options": self.http_options, "apps": {}}
        for name, a in self.apps.items():
            deps = {}
            for dname, st in a["deployments"].items():
                deps[dname] = {"spec": st.spec, "target": st.target,
                               "replicas": list(st.replicas), "retiring": list(st.retiring),
                               "version": st.version}
            state["apps"][name] = {"route_prefix": a["route_prefix"], "ingress": a["ingress"],
                                   "deployments": deps}
        try:
            from ray_amd.experimental import internal_kv

            internal_kv._internal_kv_put(CHECKPOINT_KEY, cloudpickle.dumps(state),
                                         namespace=KV_NAMESPACE)
        except Exception:  # noqa: BLE001
            pass

    async def _recover(self):
        """Re-adopt the replicas a previous incarnation started (they are named detached
        actors); ones that are gone are replaced by the reconciler."""
        data, self._recovery = self._recovery, None
        if not data:
            return
        self.http_options = data.get("http_options") or self.http_options
        for pname, attr in (("SERVE_PROXY", "proxy"), ("SERVE_GRPC_PROXY", "grpc_proxy")):
            try:
                setattr(self, attr, ray.get_actor(pname, namespace=SERVE_NAMESPACE))
            except Exception:  # noqa: BLE001
                pass
        for app_name, a in data["apps"].items():
            states = {}
            for dname, d in a["deployments"].items():
                st = _DeploymentState(app_name, d["spec"])
                st.target = d["target"]
                st.version = d["version"] + 1
                for bucket, rids in ((st.replicas, d["replicas"]), (st.retiring, d["retiring"])):
                    for rid in rids:
                        try:
                            bucket[rid] = ray.get_actor(_replica_actor_name(app_name, rid),
                                                        namespace=SERVE_NAMESPACE)
                        except Exception:  # noqa: BLE001
                            pass
                st.status = "HEALTHY" if st.replicas else "UPDATING"
                states[dname] = st
            self.apps[app_name] = {"route_prefix": a["route_prefix"], "ingress": a["ingress"],
                                   "deployments": states, "status": "DEPLOYING"}
        self.recovered = True
        self._checkpoint()
        self._notify()

    # ------------------------------------------------------------------ plumbing
    async def _ensure_loop(self):
        if self._loop_task is None:
            self._changed = asyncio.Event()
            if self._recovery:
                await self._recover()
            self._loop_task = asyncio.get_running_loop().create_task(self._control_loop())

    def _spawn(self, coro):
        t = asyncio.get_running_loop().create_task(coro)
        self._bg.add(t)
        t.add_done_callback(self._bg.discard)
        return t

    def _notify(self):
        if self._changed is not None:
            self._changed.set()
            self._changed = asyncio.Event()

    def _bump(self, st):
        st.version += 1
        self._notify()

    async def ready(self):
        await self._ensure_loop()
        return True

    # ------------------------------------------------------------------ deploy / delete
    async def deploy_application(self, app_name, route_prefix, ingress, deployments,
                                 timeout_s=120.0):
        await self._ensure_loop()
        old = self.apps.get(app_name)
        states = {}
        for spec in deployments:
            if old and spec["name"] in old["deployments"]:
                st = old["deployments"][spec["name"]]
                code_changed = st.spec.get("code_version") != spec.get("code_version")
                cfg_changed = st.spec.get("user_config") != spec.get("user_config")
                st.spec = spec
                st.start_failures = 0
                if not spec.get("autoscaling_config"):
                    st.target = spec["num_replicas"]
                if code_changed:
                    # rolling update: the old replicas keep serving until the new ones
                    # pass their health check, then drain (reference:
                    # deployment_state.py version-mismatched replicas)
                    st.retiring.update(st.replicas)
                    st.replicas = {}
                    for rid, h in list(st.starting.items()):
                        self._spawn(self._kill_replica(st, rid, h))
                    st.starting = {}
                    st.status = "UPDATING"
                elif cfg_changed and spec.get("user_config") is not None:
                    await asyncio.gather(*[r.reconfigure.remote(spec["user_config"])
                                           for r in st.replicas.values()])
            else:
                st = _DeploymentState(app_name, spec)
            states[spec["name"]] = st
        if old:
            for name, st in old["deployments"].items():
                if name not in states:
                    self._stop_all(st)
        self.apps[app_name] = {"route_prefix": route_prefix, "ingress": ingress,
                               "deployments": states, "status": "DEPLOYING"}
        self._checkpoint()
        self._reconcile()
        await self._push_routes(app_name)
        # wait for THIS app only; the control loop keeps serving everything else
        deadline = time.time() + timeout_s
        while time.time() < deadline:
            a = self.apps.get(app_name)
            if a is None or a["status"] in ("RUNNING", "DEPLOY_FAILED"):
                break
            await asyncio.sleep(0.02)
        await self._push_routes(app_name)
        return True

    async def _push_routes(self, app_name):
        self._notify()
        if self.proxy is not None:
            try:
                await self.proxy.invalidate_routes.remote(app_name)
            except Exception:  # noqa: BLE001
                pass

    async def delete_application(self, app_name):
        await self._ensure_loop()
        app = self.apps.pop(app_name, None)
        if app:
            waits = []
            for st in list(app["deployments"].values()):
                waits += self._stop_all(st)
            self._checkpoint()
            await self._push_routes(app_name)
            if waits:
                await asyncio.gather(*waits, return_exceptions=True)
        return True

    def _stop_all(self, st):
        tasks = []
        for bucket in (st.retiring, st.replicas, st.starting):
            for rid, h in list(bucket.items()):
                bucket.pop(rid, None)
                tasks.append(self._spawn(self._drain_and_kill(st, rid, h)))
        self._bump(st)
        return tasks

    # ------------------------------------------------------------------ replicas
    def _start_replica(self, st):
        spec = st.spec
        from ray_amd.serve._replica import Replica

        rid = f"{st.name}#{uuid.uuid4().hex[:6]}"
        opts = self._sched.actor_options(st, rid)
        opts["max_concurrency"] = max(100, spec.get("max_ongoing_requests", 100) * 2)
        opts["name"] = _replica_actor_name(st.app, rid)
        opts["namespace"] = SERVE_NAMESPACE
        opts["lifetime"] = "detached"
        cls = ray.remote(Replica)
        h = cls.options(**opts).remote(st.name, st.app, spec["callable"], spec["init_args"],
                                       spec["init_kwargs"], spec.get("user_config"), rid,
                                       spec["is_function"], spec.get("asgi_app"))
        if spec.get("logging_config"):  # ordered before the controller's health checks
            h.set_logging.remote(spec["logging_config"])
        st.starting[rid] = h
        self._spawn(self._await_started(st, rid, h))
        return rid

    async def _await_started(self, st, rid, h):
        """Constructor + first health check, off the control loop."""
        timeout = max(st.hc_timeout(), 60.0)
        try:
            await asyncio.wait_for(h.check_health.remote(), timeout)
        except BaseException as e:  # noqa: BLE001
            if st.starting.pop(rid, None) is None:
                return
            st.start_failures += 1
            st.error = repr(e)
            st.status = "UNHEALTHY"
            self._spawn(self._kill_replica(st, rid, h))
            self._update_app_status()
            return
        if st.starting.pop(rid, None) is None:
            return  # stopped while starting
        st.replicas[rid] = h
        st.hc[rid] = (time.time(), None, 0)
        st.start_failures = 0
        st.error = None
        if len(st.replicas) >= st.target and not st.starting:
            st.status = "HEALTHY"
            if st.retiring:
                old, st.retiring = st.retiring, {}
                for orid, oh in old.items():
                    self._spawn(self._drain_and_kill(st, orid, oh))
        self._bump(st)
        self._checkpoint()
        self._update_app_status()

    async def _drain_and_kill(self, st, rid, h):
        try:
            await asyncio.wait_for(
                h.prepare_for_shutdown.remote(st.spec.get("graceful_shutdown_wait_loop_s", 2.0)),
                st.spec.get("graceful_shutdown_timeout_s", 5))
        except BaseException:  # noqa: BLE001
            pass
        await self._kill_replica(st, rid, h)

    async def _kill_replica(self, st, rid, h):
        try:
            ray.kill(h)
        except Exception:  # noqa: BLE001
            pass
        st.hc.pop(rid, None)
        st.load.pop(rid, None)
        st.node_of.pop(rid, None)
        pg = st.pgs.pop(rid, None)
        if pg is not None:
            try:
                from ray_amd.util.placement_group import remove_placement_group

                remove_placement_group(pg)
            except Exception:  # noqa: BLE001
                pass

    def _reconcile(self):
        """Start / stop replicas toward each deployment's target. Non-blocking: starts
        are awaited by background tasks."""
        changed = False
        for app in list(self.apps.values()):
            for st in list(app["deployments"].values()):
                if st.start_failures >= MAX_START_FAILURES:
                    continue  # DEPLOY_FAILED until redeployed
                have = len(st.replicas) + len(st.starting)
                diff = st.target - have
                if diff > 0:
                    for _ in range(diff):
                        self._start_replica(st)
                    st.status = "UPDATING"
                    changed = True
                elif diff < 0:
                    n = -diff
                    for rid in list(st.starting)[:n]:
                        h = st.starting.pop(rid)
                        self._spawn(self._kill_replica(st, rid, h))
                        n -= 1
                    for rid in list(st.replicas)[:n]:
                        h = st.replicas.pop(rid)
                        self._spawn(self._drain_and_kill(st, rid, h))
                    self._bump(st)
                    changed = True
                elif not st.starting and st.status != "UNHEALTHY":
                    st.status = "HEALTHY"
        if changed:
            self._checkpoint()
        self._update_app_status()

    def _update_app_status(self):
        for app in self.apps.values():
            sts = list(app["deployments"].values())
            if any(st.start_failures >= MAX_START_FAILURES or
                   (st.start_failures and not st.replicas) for st in sts):
                app["status"] = "DEPLOY_FAILED"
            elif all(st.status == "HEALTHY" and len(st.replicas) >= st.target for st in sts):
                app["status"] = "RUNNING"
            elif app["status"] != "DEPLOY_FAILED":
                app["status"] = "DEPLOYING"

    # ------------------------------------------------------------------ health / load
    def _health_tick(self, now):
        for app in list(self.apps.values()):
            for st in list(app["deployments"].values()):
                for rid, h in list(st.replicas.items()):
                    last, task, fails = st.hc.get(rid, (0.0, None, 0))
                    if task is None and now - last >= st.period():
                        t = self._spawn(self._check_one(st, rid, h))
                        st.hc[rid] = (now, t, fails)

    async def _check_one(self, st, rid, h):
        try:
            await asyncio.wait_for(h.check_health.remote(), st.hc_timeout())
            ok = True
        except BaseException:  # noqa: BLE001
            ok = False
        last, _, fails = st.hc.get(rid, (time.time(), None, 0))
        if ok:
            st.hc[rid] = (last, None, 0)
            return
        # reference: a replica failing its health check is stopped and replaced
        if st.replicas.pop(rid, None) is not None:
            st.hc.pop(rid, None)
            self._bump(st)
            self._checkpoint()
            await self._kill_replica(st, rid, h)

    def _load_tick(self, now):
        for app in list(self.apps.values()):
            for st in list(app["deployments"].values()):
                if not st.spec.get("autoscaling_config"):
                    continue
                for rid, h in list(st.replicas.items()):
                    if rid not in st.load_tasks:
                        st.load_tasks[rid] = self._spawn(self._probe_load(st, rid, h))

    async def _probe_load(self, st, rid, h):
        try:
            v = await asyncio.wait_for(h.num_ongoing.remote(), 2.0)
            st.load[rid] = (v, time.time())
        except BaseException:  # noqa: BLE001
            pass
        finally:
            await asyncio.sleep(0.05)
            st.load_tasks.pop(rid, None)

    def record_handle_metrics(self, app_name, deployment_name, handle_id, queued, ts=None):
        """Handles push the requests they hold back (waiting for a replica slot); the
        autoscaler adds them to the replicas' ongoing requests (reference: handle metrics
        pushed to the controller, serve/config.py:54 look_back_period_s)."""
        a = self.apps.get(app_name)
        if a is None or deployment_name not in a["deployments"]:
            return False
        a["deployments"][deployment_name].handle_queued[handle_id] = (int(queued), time.time())
        return True

    def _autoscale(self, now):
        for app in list(self.apps.values()):
            for st in list(app["deployments"].values()):
                asc = st.spec.get("autoscaling_config")
                if not asc or not st.replicas:
                    continue
                fresh = 2.0
                ongoing = sum(v for rid, (v, t) in st.load.items()
                              if rid in st.replicas and now - t < fresh)
                queued = sum(q for q, t in st.handle_queued.values() if now - t < fresh)
                st.samples.append((now, ongoing + queued))
                look = float(asc.get("look_back_period_s", 30.0))
                while st.samples and now - st.samples[0][0] > look:
                    st.samples.popleft()
                avg = sum(v for _, v in st.samples) / len(st.samples)
                cur = len(st.replicas) + len(st.starting)
                # the decision itself is the deployment's policy (serve/autoscaling_policy.py;
                # reference: AutoscalingConfig._policy), called with the reference's kwargs
                st.policy_state["now"] = now
                try:
                    policy = resolve_policy(asc.get("policy"))
                    desired = int(policy(
                        curr_target_num_replicas=cur, total_num_requests=avg,
                        num_running_replicas=len(st.replicas), config=asc,
                        capacity_adjusted_min_replicas=asc.get("min_replicas", 1),
                        capacity_adjusted_max_replicas=asc.get("max_replicas", 10),
                        policy_state=st.policy_state))
                except Exception as e:  # noqa: BLE001 - a broken user policy: keep serving
                    st.error = f"autoscaling policy failed: {e!r}"
                    continue
                desired = max(asc.get("min_replicas", 1), min(asc.get("max_replicas", 10),
                                                              desired))
                if desired != cur:
                    st.target = desired
                if st.policy_state.pop("reset_samples", False):
                    st.samples.clear()

    # ------------------------------------------------------------------ per-node proxies
    def _proxy_tick(self, now):
        """ProxyLocation.EveryNode (reference: serve/_private/proxy_state.py:533,608
        ProxyStateManager.update): one HTTP proxy per alive node, pinned to it by a hard
        node-affinity strategy, started when a node joins and dropped when it dies. The
        head node's proxy is the one serve.start() created ("SERVE_PROXY"). Proxies of
        nodes that share the head's address (a one-machine cluster) listen on port + i so
        they do not collide; ``get_proxies`` reports every node's (host, port)."""
        opts = self.http_options or {}
        if opts.get("location") != "EveryNode" or self.proxy is None:
            return
        if now - getattr(self, "_proxy_checked", 0.0) < PROXY_TICK_S:
            return
        self._proxy_checked = now
        nodes = {n["NodeID"]: n for n in ray.nodes() if n.get("Alive")}
        head = next((nid for nid, n in nodes.items() if n.get("is_head_node")), None)
        head_addr = nodes[head]["NodeManagerAddress"] if head in nodes else "127.0.0.1"
        table = self.__dict__.setdefault("node_proxies", {})
        if head is not None and head not in table:
            table[head] = (self.proxy, opts.get("host", "127.0.0.1"), opts.get("port", 8000))
        for nid in [nid for nid in table if nid not in nodes]:  # node died / left
            actor = table.pop(nid)[0]
            if actor is not self.proxy:
                try:
                    ray.kill(actor)
                except Exception:  # noqa: BLE001
                    pass
        from ray_amd.serve._proxy import HTTPProxy
        from ray_amd.util.scheduling_strategies import NodeAffinitySchedulingStrategy

        for nid, n in nodes.items():
            if nid in table:
                continue
            shared = n.get("NodeManagerAddress") == head_addr
            used = {port for _, _, port in table.values()}
            port = int(opts.get("port", 8000))
            while shared and port in used:
                port += 1
            host = opts.get("host", "127.0.0.1")
            actor = ray.remote(HTTPProxy).options(
                num_cpus=0, max_concurrency=1000, name=f"SERVE_PROXY:{nid}",
                namespace=SERVE_NAMESPACE, lifetime="detached",
                scheduling_strategy=NodeAffinitySchedulingStrategy(nid, soft=False)).remote(
                host, port, opts.get("request_timeout_s"))
            table[nid] = (actor, host, port)

    async def get_proxies(self):
        """{node_id: {"host", "port", "ready"}} of the running HTTP proxies."""
        out = {}
        for nid, (actor, host, port) in list(self.__dict__.get("node_proxies", {}).items()):
            try:
                ok = await asyncio.wait_for(actor.ping.remote(), 5.0) == "ok"
            except Exception:  # noqa: BLE001
                ok = False
            out[nid] = {"host": host, "port": port, "ready": ok}
        if not out and self.proxy is not None:
            o = self.http_options or {}
            out["head"] = {"host": o.get("host", "127.0.0.1"), "port": o.get("port", 8000),
                           "ready": True}
        return out

    async def _control_loop(self):
        while True:
            try:
                now = time.time()
                self._load_tick(now)
                self._autoscale(now)
                self._reconcile()
                self._health_tick(now)
                self._proxy_tick(now)
            except Exception:  # noqa: BLE001
                import traceback

                traceback.print_exc()
            await asyncio.sleep(TICK_S)

    # ------------------------------------------------------------------ reads
    def _replica_info(self, app_name, deployment_name):
        app = self.apps.get(app_name)
        if app is None or deployment_name not in app["deployments"]:
            return None
        st = app["deployments"][deployment_name]
        # during a rolling update the old version serves until the new one is up
        reps = st.replicas if st.replicas or not st.retiring else st.retiring
        return (st.version, list(reps.items()), st.spec.get("max_ongoing_requests", 100),
                st.spec.get("max_queued_requests", -1))

    async def get_replicas(self, app_name, deployment_name):
        await self._ensure_loop()
        return self._replica_info(app_name, deployment_name)

    async def long_poll(self, snapshot: dict, timeout_s: float = 10.0):
        """Block until the replica set of any deployment in ``snapshot`` (key
        "app/deployment" -> version the caller holds) changes, then return the new infos
        (None for a deleted deployment); {} after ``timeout_s`` with no change (reference:
        long_poll.py:173 LongPollHost.listen_for_change)."""
        await self._ensure_loop()
        deadline = time.time() + timeout_s
        while True:
            out = {}
            for key, ver in snapshot.items():
                app, _, dep = key.partition("/")
                info = self._replica_info(app, dep)
                if info is None:
                    if ver is not None and ver >= 0:
                        out[key] = None
                elif info[0] != ver:
                    out[key] = info
            left = deadline - time.time()
            if out or left <= 0:
                return out
            ev = self._changed
            try:
                await asyncio.wait_for(ev.wait(), left)
            except asyncio.TimeoutError:
                pass

    async def get_routes(self):
        await self._ensure_loop()
        return {a["route_prefix"]: (name, a["ingress"]) for name, a in self.apps.items()
                if a["route_prefix"] is not None}

    async def get_ingress(self, app_name):
        await self._ensure_loop()
        a = self.apps.get(app_name)
        return None if a is None else a["ingress"]

    async def status(self):
        await self._ensure_loop()
        out = {}
        for name, a in self.apps.items():
            deps = {}
            for d, st in a["deployments"].items():
                deps[d] = {"status": st.status, "replica_states":
                           {"RUNNING": len(st.replicas), "STARTING": len(st.starting)},
                           "target_num_replicas": st.target}
                if st.error:
                    deps[d]["message"] = st.error
            out[name] = {"status": a["status"], "route_prefix": a["route_prefix"],
                         "deployments": deps}
        return out

    def get_http_options(self):
        return self.http_options

    async def shutdown(self):
        for name in list(self.apps):
            await self.delete_application(name)
        for actor, _, _ in list(self.__dict__.get("node_proxies", {}).values()):
            if actor is not self.proxy:
                try:
                    ray.kill(actor)
                except Exception:  # noqa: BLE001
                    pass
        for p in (self.proxy, self.grpc_proxy):
            if p is not None:
                try:
                    ray.kill(p)
                except Exception:  # noqa: BLE001
                    pass
        try:
            from ray_amd.experimental import internal_kv

            internal_kv._internal_kv_del(CHECKPOINT_KEY, namespace=KV_NAMESPACE)
        except Exception:  # noqa: BLE001
            pass
        return True

    def set_proxy(self, proxy, http_options=None):
        self.proxy = proxy
        if http_options:
            self.http_options = http_options
        self._checkpoint()
        return True

    def get_proxy(self):
        return self.proxy

    def set_grpc_proxy(self, proxy):
        self.grpc_proxy = proxy
        return True

    def get_grpc_proxy(self):
        return self.grpc_proxy
