"""Algorithm base (reference: rllib/algorithms/algorithm.py).

Owns the EnvRunner actors (CPU sampling), the LearnerGroup (GPU learning) and
the train()/save()/restore()/evaluate() lifecycle; subclasses implement
``training_step``."""

from __future__ import annotations

import os
import pickle
import time

import numpy as np

import ray_amd as ray
from ray_amd.rllib.env.env_runner import SingleAgentEnvRunner
from ray_amd.rllib.env.envs import make_env


class PerModuleLearners:
    """Multi-agent off-policy learners (DQN, SAC): one learner per module built by
    ``make(obs_space, action_space)``; only the ``trainable`` ones are updated. The
    algorithm keeps one replay buffer per trainable module."""

    def __init__(self, make, specs, trainable=None):
        self.make = make
        self.learners = {mid: self._make(mid, os_, as_) for mid, (os_, as_) in specs.items()}
        self.trainable = set(trainable) if trainable else set(specs)

    def _make(self, mid, os_, as_):
        import inspect

        try:
            n = len(inspect.signature(self.make).parameters)
        except (TypeError, ValueError):
            n = 2
        return self.make(os_, as_, mid) if n >= 3 else self.make(os_, as_)

    def add(self, mid, spec, trainable=True):
        """A new module's learner(s) mid-training (Algorithm.add_module)."""
        self.learners[mid] = self._make(mid, spec[0], spec[1])
        if trainable:
            self.trainable.add(mid)

    def remove(self, mid):
        lr = self.learners.pop(mid, None)
        self.trainable.discard(mid)
        if lr is not None:
            lr.shutdown()

    # reference-named module-set API (learner_group.py:494 add_module, :520 remove_module,
    # get/set_module_state, get/set_optimizer_state): here each module has its own learner
    # (group), built by ``make`` — the off-policy algorithms keep one replay buffer and one
    # target network per module
    def add_module(self, *, module_id, module_spec, config_overrides=None,
                   new_should_module_be_updated=None):
        spec = tuple(module_spec) if isinstance(module_spec, (tuple, list)) else \
            (module_spec.observation_space, module_spec.action_space)
        self.add(module_id, spec)
        if new_should_module_be_updated is not None:
            ids = list(self.learners)
            f = new_should_module_be_updated
            self.trainable = {m for m in ids if f(m)} if callable(f) else set(f) & set(ids)
        return list(self.learners)

    def remove_module(self, module_id, *, new_should_module_be_updated=None):
        self.remove(module_id)
        return list(self.learners)

    def get_module_state(self, module_ids=None) -> dict:
        ids = list(self.learners) if module_ids is None else \
            [m for m in module_ids if m in self.learners]
        return {m: self.learners[m].get_weights() for m in ids}

    def set_module_state(self, state: dict):
        for m, w in state.items():
            self.learners[m].set_weights(w)

    def get_optimizer_state(self) -> dict:
        """{module_id: that module's optimizer states} (each learner group holds one)."""
        return {m: lr.get_optimizer_state()[m] for m, lr in self.learners.items()}

    def set_optimizer_state(self, state: dict):
        for m, st in state.items():
            self.learners[m].set_optimizer_state({m: st})

    def sync_target(self):
        for mid in self.trainable:
            getattr(self.learners[mid], "sync_target", lambda: None)()

    def get_weights(self):
        return {mid: lr.get_weights() for mid, lr in self.learners.items()}

    def set_weights(self, w):
        for mid, wm in w.items():
            if mid in self.learners:
                self.learners[mid].set_weights(wm)

    def get_state(self):
        return {mid: lr.get_state() for mid, lr in self.learners.items()}

    def set_state(self, s):
        for mid, st in s.items():
            self.learners[mid].set_state(st)

    def shutdown(self):
        for lr in self.learners.values():
            lr.shutdown()


def flat_transitions(b: dict, keys=("obs", "next_obs", "actions", "rewards", "terminateds")):
    """[T, B] runner fragment -> transition rows for a replay buffer; padding rows
    (loss_mask 0, batch_mode="complete_episodes") are dropped."""
    T, B = b["rewards"].shape
    flat = {k: b[k].reshape((T * B,) + b[k].shape[2:]) for k in keys}
    if "loss_mask" in b:
        keep = b["loss_mask"].reshape(-1) > 0
        flat = {k: v[keep] for k, v in flat.items()}
    return flat


def add_agent_rows(buffers, batch):
    """Completed agent rows (loss_mask 1) of a multi-agent sample become transitions of
    their module's replay buffer; returns the number added."""
    n = 0
    for mid, mb in batch["modules"].items():
        if mid not in buffers:
            continue
        real = mb["loss_mask"] == 1
        if real.any():
            buffers[mid].add({k: mb[k][real] for k in
                              ("obs", "next_obs", "actions", "rewards", "terminateds")})
            n += int(real.sum())
    return n


class Algorithm:
    kind = "ppo"
    supports_multi_agent = False

    def __init__(self, config):
        if not ray.is_initialized():
            ray.init()
        self.config = config
        self.cfg = config.to_dict()
        self.cfg["module_kind"] = getattr(self, "module_kind", "actor_critic")
        mcfg = self.cfg.get("model") or {}
        if isinstance(mcfg.get("custom_model"), str):
            # the driver's ModelCatalog registration travels with the config to the
            # runner and learner processes (reference: the registry in the GCS KV)
            from ray_amd.rllib.models import ModelCatalog

            cls = ModelCatalog._custom_models.get(mcfg["custom_model"])
            if cls is not None:
                self.cfg["model"] = dict(mcfg, custom_model=cls)
        if type(self).validate_env is not Algorithm.validate_env:  # overridden: runners call it
            self.cfg["_validate_env"] = type(self).validate_env
        if config.env is None and config.observation_space is not None and \
                config.action_space is not None:
            # no local env (external simulators via PolicyServerInput, or offline data):
            # the spaces come from the config
            import types

            probe = types.SimpleNamespace(observation_space=config.observation_space,
                                          action_space=config.action_space,
                                          close=lambda: None)
        else:
            probe = make_env(config.env, config.env_config)
        self.observation_space = probe.observation_space
        self.action_space = probe.action_space
        # the modules see the env-to-module connector pipeline's output space; a
        # learner-side MeanStdFilter keeps its statistics on the learner (HIP kernel)
        from ray_amd.rllib.callbacks import MetricsLogger, make_callbacks
        from ray_amd.rllib.connectors.connector_v2 import build_pipeline

        pipe = build_pipeline(config.env_to_module_connector, self.observation_space,
                              self.action_space)
        learner_filter = config.observation_filter == "MeanStdFilter" or any(
            getattr(c, "learner_side", False) for c in pipe.connectors)
        self.cfg["_learner_obs_filter"] = learner_filter
        self.observation_space = pipe.observation_space
        self.callbacks = make_callbacks(config.callbacks_class)
        self.metrics = MetricsLogger()
        self._custom_metrics = {}
        self.is_multi_agent = bool(getattr(config, "is_multi_agent", False))
        self.cfg["is_multi_agent"] = self.is_multi_agent
        if self.is_multi_agent and not self.supports_multi_agent:
            raise NotImplementedError(f"{type(self).__name__} does not support multi-agent "
                                      "configs yet (PPO does)")
        if self.is_multi_agent:
            self.module_specs = self._module_specs(config, probe)
            self.cfg["_module_specs"] = self.module_specs
        probe.close()
        self.iteration = 0
        self.total_env_steps = 0
        self.weights_version = 0
        self._episode_returns = []
        self._episode_lengths = []
        self._module_returns = {}
        self._t_start = time.time()
        nr = int(config.num_env_runners)
        local_cls = getattr(self, "env_runner_cls", None) or SingleAgentEnvRunner
        if self.is_multi_agent:
            from ray_amd.rllib.env.multi_agent_env_runner import MultiAgentEnvRunner

            local_cls = MultiAgentEnvRunner
        self._runner_cls = local_cls
        runner_cls = ray.remote(local_cls)
        opts = {"num_cpus": config.num_cpus_per_env_runner}
        if config.num_gpus_per_env_runner:
            opts["num_gpus"] = config.num_gpus_per_env_runner
        self._runner_remote_cls, self._runner_opts = runner_cls, opts
        from ray_amd.rllib.utils.actor_manager import FaultTolerantActorManager

        # EnvRunners behind a FaultTolerantActorManager (reference: actor_manager.py:193,
        # AlgorithmConfig.fault_tolerance): a dead runner is recreated with the same
        # worker index and the current weights, or dropped (ignore_env_runner_failures)
        self._runners = FaultTolerantActorManager(restore_fn=self._restore_runner)
        self._last_weights_ref = None
        self._policy_server = None
        self._policy_server_local = None
        if nr > 0 and float(getattr(config, "num_gpus_per_policy_server", 0) or 0) > 0:
            self._start_policy_server(config, nr, probe)
        if nr > 0:
            rs = [runner_cls.options(**opts).remote(self.cfg, i + 1) for i in range(nr)]
            ray.get([r.ping.remote() for r in rs])
            self._runners.add_actors(rs)
            self.local_runner = None
        else:
            self.local_runner = local_cls(self.cfg, 0)
        # evaluation EnvRunners (evaluation_num_env_runners): exploration off, the
        # evaluation_config overrides, run beside training (evaluation_parallel_to_training)
        self._eval_runners = []
        self._eval_local = None
        self._eval_pending = None
        ne = int(getattr(config, "evaluation_num_env_runners", 0) or 0)
        if ne > 0:
            ecfg = dict(self.cfg)
            ecfg.pop("_policy_server", None)  # evaluation runners infer locally
            ecfg.update(dict(getattr(config, "evaluation_config", None) or {}))
            ecfg["_record_episodes"] = False
            self._eval_cfg = ecfg
            self._eval_runners = [runner_cls.options(**opts).remote(ecfg, 1000 + i)
                                  for i in range(ne)]
            ray.get([r.ping.remote() for r in self._eval_runners])
        self.setup()
        self.callbacks.on_algorithm_init(algorithm=self, metrics_logger=self.metrics)

    @staticmethod
    def _module_specs(config, probe):
        """{module_id: (observation_space, action_space)}; spaces not given in ``policies``
        come from the first agent ``policy_mapping_fn`` routes to that module."""
        from ray_amd.rllib.env.multi_agent_env_runner import DEFAULT_MODULE_ID, _default_mapping

        pols = config.policies
        ids = list(pols) if not isinstance(pols, dict) else list(pols.keys())
        ids = ids or [DEFAULT_MODULE_ID]
        fn = config.policy_mapping_fn or _default_mapping
        agents = sorted(probe.get_agent_ids(), key=str) if hasattr(probe, "get_agent_ids") \
            else []
        specs = {}
        for mid in ids:
            spec = pols.get(mid) if isinstance(pols, dict) else None
            os_ = getattr(spec, "observation_space", None) or \
                (spec[0] if isinstance(spec, (tuple, list)) and len(spec) >= 2 else None)
            as_ = getattr(spec, "action_space", None) or \
                (spec[1] if isinstance(spec, (tuple, list)) and len(spec) >= 2 else None)
            if os_ is None or as_ is None:
                aid = next((a for a in agents if fn(a, None) == mid), agents[0] if agents
                           else None)
                os_ = os_ or (probe.get_observation_space(aid) if aid is not None
                              else probe.observation_space)
                as_ = as_ or (probe.get_action_space(aid) if aid is not None
                              else probe.action_space)
            specs[mid] = (os_, as_)
        return specs

    def setup(self):
        pass

    # ---------------------------------------------------------------- env runner group
    @property
    def env_runners(self):
        """The healthy EnvRunner actors."""
        return self._runners.actors()

    @env_runners.setter
    def env_runners(self, runners):
        from ray_amd.rllib.utils.actor_manager import FaultTolerantActorManager

        self._runners = FaultTolerantActorManager(restore_fn=self._restore_runner)
        self._runners.add_actors(list(runners or []))

    def _restore_runner(self, actor_id):
        cfg = self.config
        if self._runners.num_restarts >= cfg.max_num_env_runner_restarts:
            return None
        if cfg.delay_between_env_runner_restarts_s:
            time.sleep(cfg.delay_between_env_runner_restarts_s)
        r = self._runner_remote_cls.options(**self._runner_opts).remote(self.cfg, actor_id)
        ray.get(r.ping.remote())
        w = self._last_weights_ref
        if w is None:
            w = ray.put(self._weights_for_runners())
        ray.get(r.set_weights.remote(w, self.weights_version))
        return r

    def _weights_for_runners(self):
        return self.learner_group.get_weights()

    def _foreach_runner(self, fn):
        """fn(runner) -> ObjectRef on every healthy EnvRunner; results of the ones that
        answered. Dead runners are handled per AlgorithmConfig.fault_tolerance."""
        res = self._runners.foreach_actor(fn)
        bad = [r for r in res if not r.ok]
        if bad:
            self._on_runner_failures(bad)
        return [r.value for r in res if r.ok]

    def _on_runner_failures(self, bad):
        from ray_amd.rllib.utils.actor_manager import _is_actor_failure

        app = [r for r in bad if not _is_actor_failure(r.value)]
        if app:  # an exception inside the runner (env / user code): not a lost actor
            raise app[0].value
        cfg = self.config
        if cfg.restart_failed_env_runners:
            self.restore_env_runners()
        elif not cfg.ignore_env_runner_failures:
            raise bad[0].value
        if self._runners.num_healthy_actors() == 0:
            raise RuntimeError("no healthy EnvRunner left (all failed; restart disabled or "
                               "max_num_env_runner_restarts reached)")

    def restore_env_runners(self):
        """Probe unhealthy EnvRunners; recreate dead ones (reference:
        Algorithm.restore_env_runners / EnvRunnerGroup.probe_unhealthy_env_runners)."""
        restored = self._runners.probe_unhealthy_actors(
            self.config.env_runner_health_probe_timeout_s,
            restore=self.config.restart_failed_env_runners)
        return restored

    @property
    def num_env_runner_restarts(self):
        return self._runners.num_restarts

    def _start_policy_server(self, config, nr, probe):
        """One batched GPU inference process for all runners (rllib/env/policy_server.py):
        discrete actor-critic modules whose observations reach the module unchanged."""
        import functools

        from ray_amd.rllib.core.rl_module.rl_module import build_module
        from ray_amd.rllib.env.policy_server import PolicyServer

        if self.cfg.get("module_kind", "actor_critic") != "actor_critic" or \
                not hasattr(probe.action_space, "n") or self.is_multi_agent or \
                self.cfg.get("env_to_module_connector") or \
                self.cfg.get("observation_filter", "NoFilter") not in (None, "NoFilter"):
            raise ValueError("num_gpus_per_policy_server needs a single-agent discrete "
                             "actor-critic module fed the raw observations")
        fn = functools.partial(build_module, dict(self.cfg), probe.observation_space,
                               probe.action_space)
        B = int(config.num_envs_per_env_runner)
        args = (fn, nr, B, tuple(probe.observation_space.shape), int(probe.action_space.n))
        import torch

        if int(getattr(config, "num_learners", 0) or 0) == 0 and torch.cuda.is_available():
            # local learner: the server thread lives in this process and shares the
            # learner's GPU context (its own stream; graph captures take turns through
            # ops.graph_lock) — no second process time-slicing the GPU with the learner
            self._policy_server_local = PolicyServer(*args)
            self.cfg["_policy_server"] = self._policy_server_local.mailbox()
            return
        srv = ray.remote(PolicyServer).options(
            num_gpus=float(config.num_gpus_per_policy_server), num_cpus=1).remote(*args)
        self._policy_server = srv
        self.cfg["_policy_server"] = ray.get(srv.mailbox.remote())

    # ---------------------------------------------------------------- weights
    def _sync_weights(self, weights):
        self.weights_version += 1
        if self._policy_server is not None:
            self._policy_server.set_weights.remote(weights, self.weights_version)
        if getattr(self, "_policy_server_local", None) is not None:
            self._policy_server_local.set_weights(weights, self.weights_version)
        if self._runners.num_actors():
            ref = ray.put(weights)
            self._last_weights_ref = ref
            self._foreach_runner(lambda r: r.set_weights.remote(ref, self.weights_version))
        else:
            self.local_runner.set_weights(weights, self.weights_version)

    def _take_metrics(self, batch):
        """Metrics that came back attached to a sample (async sampling paths)."""
        m = batch.pop("_metrics", None) if isinstance(batch, dict) else None
        if m is not None:
            self.__dict__.setdefault("_async_ms", []).append(m)

    def _collect_metrics(self):
        if getattr(self, "_metrics_from_samples", False) and self.env_runners:
            ms, self._async_ms = self.__dict__.get("_async_ms", []), []
        elif self._runners.num_actors():
            ms = self._foreach_runner(lambda r: r.get_metrics.remote())
        else:
            ms = [self.local_runner.get_metrics()]
        cm = {}
        for m in ms:
            self._episode_returns.extend(m["episode_returns"])
            self._episode_lengths.extend(m["episode_lengths"])
            for k, v in (m.get("custom_metrics") or {}).items():
                cm.setdefault(k, []).append(v)
            for mid, rs in m.get("module_episode_returns", {}).items():
                self._module_returns.setdefault(mid, []).extend(rs)
        self._custom_metrics = {k: float(np.mean(v)) for k, v in cm.items()}
        k = self.config.metrics_num_episodes_for_smoothing
        self._episode_returns = self._episode_returns[-k:]
        self._episode_lengths = self._episode_lengths[-k:]
        self._module_returns = {mid: r[-k:] for mid, r in self._module_returns.items()}

    # ---------------------------------------------------------------- train loop
    def train(self) -> dict:
        t0 = time.time()
        steps0 = self.total_env_steps
        if self.config.restart_failed_env_runners and self._runners.num_actors() and \
                self._runners.num_healthy_actors() < self._runners.num_actors():
            self.restore_env_runners()
        do_eval = bool(self.config.evaluation_interval) and \
            (self.iteration + 1) % self.config.evaluation_interval == 0
        parallel_eval = do_eval and self._eval_runners and \
            getattr(self.config, "evaluation_parallel_to_training", False)
        if parallel_eval:
            self.callbacks.on_evaluate_start(algorithm=self, metrics_logger=self.metrics)
            self._eval_pending = self._start_eval()
        res = self.training_step()
        mt = self.config.min_time_s_per_iteration
        while mt and time.time() - t0 < mt:
            r2 = self.training_step()
            res.update(r2)
        self.iteration += 1
        self._collect_metrics()
        dt = time.time() - t0
        rets = self._episode_returns
        out = {
            "training_iteration": self.iteration,
            "env_runners": {
                "episode_return_mean": float(np.mean(rets)) if rets else float("nan"),
                "episode_return_max": float(np.max(rets)) if rets else float("nan"),
                "episode_return_min": float(np.min(rets)) if rets else float("nan"),
                "episode_len_mean": float(np.mean(self._episode_lengths))
                if self._episode_lengths else float("nan"),
                "num_episodes": len(rets),
            },
            **({"module_episode_returns_mean": {
                mid: float(np.mean(r)) for mid, r in self._module_returns.items() if r}}
               if self.is_multi_agent else {}),
            "num_env_steps_sampled_lifetime": self.total_env_steps,
            "num_env_steps_sampled_this_iter": self.total_env_steps - steps0,
            "env_steps_per_sec": (self.total_env_steps - steps0) / max(dt, 1e-9),
            "time_this_iter_s": dt,
            "time_total_s": time.time() - self._t_start,
            "learners": res,
        }
        out["episode_reward_mean"] = out["env_runners"]["episode_return_mean"]
        # old-stack names used by tuned-example stop criteria (sampler_results/...,
        # timesteps_total)
        out["timesteps_total"] = self.total_env_steps
        out["sampler_results"] = {"episode_reward_mean": out["episode_reward_mean"],
                                  "episode_len_mean": out["env_runners"]["episode_len_mean"]}
        if self._custom_metrics:
            out["env_runners"]["custom_metrics"] = dict(self._custom_metrics)
            out["custom_metrics"] = dict(self._custom_metrics)
        if do_eval:
            if parallel_eval:
                out["evaluation"] = self._finish_eval(self._eval_pending)
                self._eval_pending = None
            else:
                self.callbacks.on_evaluate_start(algorithm=self, metrics_logger=self.metrics)
                out["evaluation"] = self.evaluate()
            self.callbacks.on_evaluate_end(algorithm=self, evaluation_metrics=out["evaluation"],
                                           metrics_logger=self.metrics)
        out["num_healthy_env_runners"] = self._runners.num_healthy_actors()
        out["num_env_runner_restarts"] = self._runners.num_restarts
        self.callbacks.on_train_result(algorithm=self, result=out, metrics_logger=self.metrics)
        extra = self.metrics.reduce_all()
        if extra:
            out.setdefault("custom_metrics", {}).update(extra)
        return out

    def training_step(self) -> dict:
        raise NotImplementedError

    # ---------------------------------------------------------------- Trainable surface
    # (reference: rllib/algorithms/algorithm.py — Algorithm is a tune.Trainable)
    def step(self) -> dict:
        """One training iteration (Trainable.step); ``train`` is the same call."""
        return self.train()

    def cleanup(self):
        """Trainable.cleanup: release runners, learners and the policy server."""
        self.stop()

    def log_result(self, result: dict) -> None:
        """Trainable.log_result: keep the latest result (``callbacks`` already saw it)."""
        self._last_result = result

    def get_auto_filled_metrics(self, now=None, time_this_iter=None, timestamp=None,
                                debug_metrics_only=False) -> dict:
        import datetime
        import os as _os
        import socket

        now = now or datetime.datetime.now()
        m = {"trial_id": getattr(self, "trial_id", "default"),
             "time_this_iter_s": time_this_iter,
             "time_total_s": time.time() - self._t_start,
             "training_iteration": self.iteration}
        if not debug_metrics_only:
            m.update({"date": now.strftime("%Y-%m-%d_%H-%M-%S"),
                      "timestamp": int(timestamp or time.time()),
                      "pid": _os.getpid(), "hostname": socket.gethostname(),
                      "node_ip": "127.0.0.1"})
        return m

    @classmethod
    def get_default_config(cls):
        """The AlgorithmConfig subclass whose ``algo_class`` is this algorithm."""
        from ray_amd.rllib.algorithms.algorithm_config import AlgorithmConfig

        def subs(c):
            for s_ in c.__subclasses__():
                yield s_
                yield from subs(s_)

        for sub in subs(AlgorithmConfig):
            try:
                inst = sub()
            except Exception:  # noqa: BLE001 - configs that need arguments
                continue
            if inst.algo_class is cls:
                return inst
        return AlgorithmConfig(algo_class=cls)

    @classmethod
    def get_default_policy_class(cls, config=None):
        return _PolicyView

    @classmethod
    def validate_config(cls, config) -> None:
        v = getattr(config, "validate", None)
        if callable(v):
            v()

    @staticmethod
    def merge_algorithm_configs(config1: dict, config2: dict,
                                _allow_unknown_configs: bool | None = None) -> dict:
        """Deep-merge ``config2`` into a copy of ``config1`` (reference:
        Algorithm.merge_algorithm_configs); unknown top-level keys raise unless allowed."""
        import copy

        out = copy.deepcopy(dict(config1))
        for k, v in dict(config2 or {}).items():
            if k not in out and _allow_unknown_configs is False:
                raise ValueError(f"Unknown config parameter `{k}`")
            if isinstance(v, dict) and isinstance(out.get(k), dict):
                out[k] = Algorithm.merge_algorithm_configs(out[k], v, True)
            else:
                out[k] = v
        return out

    @classmethod
    def default_resource_request(cls, config):
        """Resources one trial of this algorithm holds (Tune): the driver bundle (CPU +
        local learner GPUs), one bundle per env runner, one per remote learner."""
        from ray_amd.tune.registry import PlacementGroupFactory

        c = config if not isinstance(config, dict) else cls.get_default_config().update_from_dict(
            config)
        nl = int(getattr(c, "num_learners", 0) or 0)
        g = float(getattr(c, "num_gpus_per_learner", 0) or 0)
        head = {"CPU": 1.0}
        if nl == 0 and g:
            head["GPU"] = g
        bundles = [head]
        for _ in range(int(getattr(c, "num_env_runners", 0) or 0)):
            b = {"CPU": float(getattr(c, "num_cpus_per_env_runner", 1) or 1)}
            if getattr(c, "num_gpus_per_env_runner", 0):
                b["GPU"] = float(c.num_gpus_per_env_runner)
            bundles.append(b)
        for _ in range(nl):
            bundles.append({"CPU": 1.0, **({"GPU": g} if g else {})})
        if float(getattr(c, "num_gpus_per_policy_server", 0) or 0) > 0:
            bundles.append({"CPU": 1.0, "GPU": float(c.num_gpus_per_policy_server)})
        return PlacementGroupFactory(bundles, strategy="PACK")

    @classmethod
    def resource_help(cls, config) -> str:
        pgf = cls.default_resource_request(config)
        return (f"{cls.__name__} asks for {len(pgf.bundles)} bundles {pgf.bundles}: the "
                "driver / local learner, one per env runner (num_cpus_per_env_runner, "
                "num_gpus_per_env_runner), one per remote learner (num_gpus_per_learner).")

    def export_policy_checkpoint(self, export_dir: str, policy_id=None) -> None:
        """Policy state (weights + spaces) as a weights-only checkpoint directory."""
        import os as _os

        import torch

        _os.makedirs(export_dir, exist_ok=True)
        pol = self.get_policy(policy_id)
        torch.save({"weights": {k: torch.as_tensor(v) for k, v in pol.get_weights().items()},
                    "policy_id": policy_id or "default_policy"},
                   _os.path.join(export_dir, "policy_state.pt"))

    def import_model(self, import_file: str):
        """Load module weights exported by ``export_policy_model`` (weights-only .pt);
        Keras h5 files (``import_policy_model_from_h5``) need tensorflow."""
        import torch

        if str(import_file).endswith(".h5"):
            return self.import_policy_model_from_h5(import_file)
        sd = torch.load(import_file, weights_only=True, map_location="cpu")
        if isinstance(sd, dict) and "weights" in sd:
            sd = sd["weights"]
        self.set_weights(sd)

    def import_policy_model_from_h5(self, import_file: str, policy_id=None):
        try:
            import tensorflow  # noqa: F401
        except ImportError:
            raise ImportError("import_policy_model_from_h5 requires tensorflow (Keras h5 "
                              "weights), which is not installed") from None
        raise NotImplementedError("Keras h5 weights cannot be mapped onto torch RLModules")

    def _sample(self, total: int):
        """Synchronous parallel sampling of >= total env steps (reference:
        rllib/execution/rollout_ops.py:synchronous_parallel_sample)."""
        cfg = self.config
        per = cfg.rollout_fragment_length
        batches = []
        got = 0
        while got < total:
            if self._runners.num_actors():
                bs = self._foreach_runner(lambda r: r.sample.remote(per))
            else:
                bs = [self.local_runner.sample(per)]
            for b in bs:
                got += b["env_steps"]
            batches.extend(bs)
        self.total_env_steps += got
        return batches

    def evaluate(self) -> dict:
        """Evaluation rollouts (exploration off) over ``evaluation_duration`` episodes or
        timesteps: on the evaluation EnvRunners in parallel when
        ``evaluation_num_env_runners`` > 0, else on one local evaluation runner that is
        built once and reused (reference: algorithm.py:642,908)."""
        ope = getattr(self.config, "off_policy_estimation_methods", None)
        ev = dict(getattr(self.config, "evaluation_config", None) or {})
        if ope and (ev.get("input_") or ev.get("input")):
            # offline evaluation (reference: evaluation_config={"input": ...}): the
            # estimators run on the logged evaluation data, no env rollouts
            return {"off_policy_estimator": self.off_policy_estimates()}
        out = self._finish_eval(self._start_eval())
        if ope:
            out["off_policy_estimator"] = self.off_policy_estimates()
        return out

    def off_policy_estimates(self) -> dict:
        """Off-policy estimates of the current policy (reference: algorithm_config.py:2040
        off_policy_estimation_methods, rllib/offline/offline_evaluator.py): every
        configured estimator ({name: {"type": ImportanceSampling | "wis" | ..., kwargs}})
        on the logged data of ``evaluation_config["input_"]`` (else ``input_``), read
        through ray_amd.data. DM / DR first fit their Q-model on the same rows."""
        from ray_amd.rllib.offline import estimators as E
        from ray_amd.rllib.offline.io import read_offline_dataset

        methods = getattr(self.config, "off_policy_estimation_methods", None) or {}
        ev = dict(getattr(self.config, "evaluation_config", None) or {})
        inp = ev.get("input_") or ev.get("input") or self.config.input_
        if not inp:
            raise ValueError("off_policy_estimation_methods need logged data: "
                             "evaluation_config={'input_': path} or offline_data(input_=...)")
        if getattr(self, "_ope_batch", None) is None:
            ds = read_offline_dataset(inp, read_method=getattr(self.config,
                                                               "input_read_method", None))
            cols = {}
            for b in ds.iter_batches(batch_size=65536):
                for k, v in b.items():
                    cols.setdefault(k, []).append(np.asarray(v))
            self._ope_batch = {k: np.concatenate(v) for k, v in cols.items()}
        batch = self._ope_batch
        names = {"is": E.ImportanceSampling, "importancesampling": E.ImportanceSampling,
                 "wis": E.WeightedImportanceSampling,
                 "weightedimportancesampling": E.WeightedImportanceSampling,
                 "dm": E.DirectMethod, "directmethod": E.DirectMethod,
                 "dr": E.DoublyRobust, "doublyrobust": E.DoublyRobust}
        split = getattr(self.config, "ope_split_batch_by_episode", True)
        policy = self.get_policy()
        out = {}
        for name, spec in methods.items():
            spec = dict(spec or {})
            cls = spec.pop("type", name)
            if isinstance(cls, str):
                key = cls.rsplit(".", 1)[-1].lower()
                if key not in names:
                    raise ValueError(f"unknown off-policy estimator {cls!r}")
                cls = names[key]
            est = cls(policy, gamma=self.config.gamma, **spec)
            train_metrics = est.train(batch)
            res = est.estimate(batch, split_batch_by_episode=split)
            if train_metrics:
                res.update({f"train_{k}": v for k, v in train_metrics.items()})
            out[name] = res
        return out

    def _start_eval(self):
        w = self._weights_for_runners()
        if self._eval_runners:
            ref = ray.put(w)
            for r in self._eval_runners:
                r.set_weights.remote(ref, None)
            return {"inflight": {r.sample.remote(self.config.rollout_fragment_length,
                                                 explore=False, with_metrics=True): r
                                 for r in self._eval_runners}}
        if self._eval_local is None:
            ecfg = dict(self.cfg)
            ecfg.pop("_policy_server", None)  # evaluation runners infer locally
            ecfg.update(dict(getattr(self.config, "evaluation_config", None) or {}))
            ecfg["_record_episodes"] = False
            self._eval_local = self._runner_cls(ecfg, 999)
        self._eval_local.set_weights(w, None)
        return {"local": True}

    def _finish_eval(self, st) -> dict:
        n = int(self.config.evaluation_duration)
        by_steps = getattr(self.config, "evaluation_duration_unit", "episodes") == "timesteps"
        rets, lens, steps = [], [], 0

        def done():
            return steps >= n if by_steps else len(rets) >= n

        frag = self.config.rollout_fragment_length
        if st.get("local"):
            while not done():
                b = self._eval_local.sample(frag, explore=False)
                steps += b["env_steps"]
                m = self._eval_local.get_metrics()
                rets.extend(m["episode_returns"])
                lens.extend(m["episode_lengths"])
        else:
            inflight = st["inflight"]
            while inflight:
                ready, _ = ray.wait(list(inflight), num_returns=1)
                r = inflight.pop(ready[0])
                try:
                    b = ray.get(ready[0])
                except Exception:  # noqa: BLE001  (a dead evaluation runner: skip it)
                    continue
                steps += b["env_steps"]
                m = b.get("_metrics") or {}
                rets.extend(m.get("episode_returns", []))
                lens.extend(m.get("episode_lengths", []))
                if not done():
                    inflight[r.sample.remote(frag, explore=False, with_metrics=True)] = r
            if not done():  # every runner died: finish locally
                return self._finish_eval(self._start_eval_local_fallback())
        sel = rets if by_steps else rets[:n]
        return {"env_runners": {
            "episode_return_mean": float(np.mean(sel)) if sel else float("nan"),
            "episode_len_mean": float(np.mean(lens[:len(sel)])) if sel else float("nan"),
            "num_episodes": len(sel), "num_env_steps_sampled": steps},
            "num_evaluation_env_runners": len(self._eval_runners)}

    def _start_eval_local_fallback(self):
        self._eval_runners = []
        return self._start_eval()

    # ---------------------------------------------------------------- offline data
    def _setup_offline(self):
        """Offline algorithms (BC, MARWIL, CQL): the recorded experience as a ray_amd.data
        dataset (rllib/offline/offline_data.py)."""
        from ray_amd.rllib.offline import OfflineData

        cfg = self.config
        if not cfg.input_:
            raise ValueError(f"{type(self).__name__} is offline: set "
                             "config.offline_data(input_=<recorded experience>)")
        self.offline = OfflineData(cfg.input_, cfg.gamma, cfg.seed,
                                   read_method=getattr(cfg, "input_read_method", None),
                                   read_kwargs=getattr(cfg, "input_read_method_kwargs", None),
                                   shuffle_buffer_size=getattr(cfg, "shuffle_buffer_size",
                                                               None))
        self._offline_fed = False

    def _offline_updates(self, n_updates: int, batch_size: int, transform=None) -> dict:
        """``n_updates`` learner updates on offline batches of ``batch_size`` rows in
        total: one local learner samples the dataset's shuffled epoch stream; N learner
        actors each pull batch_size / N rows per update from their streaming_split shard
        (reference: offline_data.py sample(num_shards=N) -> update_from_iterator)."""
        lg = self.learner_group
        if getattr(lg, "remote", False):
            n = len(lg.actors)
            its = None
            if not self._offline_fed:
                its = self.offline.shards(n)
                self._offline_fed = True
            return lg.update_from_iterator(its, num_iters=n_updates,
                                           minibatch_size=max(1, batch_size // n),
                                           transform=transform, seed=self.config.seed)
        stats = {}
        for _ in range(int(n_updates)):
            b = self.offline.sample(batch_size)
            stats = lg.update_from_batch(transform(b) if transform else b)
        return stats

    # ---------------------------------------------------------------- inference
    def _new_module(self, obs_space, act_space, module_id=None):
        """An inference module of this algorithm's kind (what its EnvRunners run)."""
        kind = self.cfg.get("module_kind", "actor_critic")
        if kind == "q":
            from ray_amd.rllib.core.rl_module import QModule

            mc = dict(self.config.model or {})
            mc["dueling"] = self.cfg.get("dueling", True)
            return QModule(obs_space, act_space, mc)
        if kind == "sac":
            from ray_amd.rllib.core.rl_module import SquashedGaussianPolicy

            return SquashedGaussianPolicy(obs_space, act_space,
                                          self.cfg.get("policy_model_config") or
                                          self.config.model)
        from ray_amd.rllib.core.rl_module.rl_module import build_module

        return build_module(self.cfg, obs_space, act_space, module_id)

    def get_module(self, module_id=None):
        """The RLModule with the current weights, on the CPU, for inference (reference:
        Algorithm.get_module)."""
        if self.is_multi_agent:
            from ray_amd.rllib.env.multi_agent_env_runner import DEFAULT_MODULE_ID

            mid = module_id or DEFAULT_MODULE_ID
            os_, as_ = self.module_specs[mid]
            mods = self.__dict__.setdefault("_infer_modules", {})
            if mid not in mods:
                mods[mid] = self._new_module(os_, as_, mid)
            m = mods[mid]
            m.load_state_dict(self.get_weights()[mid])
            self._infer_filter = None
        else:
            if not hasattr(self, "_infer_module"):
                self._infer_module = self._new_module(self.observation_space,
                                                      self.action_space)
            m = self._infer_module
            w = dict(self.get_weights())
            cs = w.pop("__connector_state__", None)
            m.load_state_dict(w)
            self._infer_filter = None
            if cs is not None:  # same normalization the EnvRunners apply
                from ray_amd.ops.functional import RunningMeanStd

                f = RunningMeanStd(tuple(cs["mean"].shape))
                f.load_state_dict(cs)
                self._infer_filter = f
        m.eval()
        return m

    def compute_single_action(self, obs, explore=False, policy_id=None):
        import torch

        m = self.get_module(policy_id)
        if self._infer_filter is not None:
            obs = self._infer_filter.normalize(
                torch.as_tensor(np.asarray(obs, np.float32))).numpy()
        kind = self.cfg.get("module_kind", "actor_critic")
        with torch.no_grad():
            x = torch.as_tensor(np.asarray(obs)[None])
            if kind == "q":
                a = m(x.float()).argmax(-1)
                if explore and np.random.random() < getattr(self, "epsilon", 0.0):
                    a = torch.tensor([np.random.randint(self.action_space.n)])
            elif kind == "sac":
                a, _ = m(x.float(), explore)
                a = a.float()
            else:
                di = m.forward_inference(x)["action_dist_inputs"]
                a, _ = m.sample_actions(di, explore)
        a = a[0].numpy()
        return int(a) if a.ndim == 0 else a

    def compute_actions(self, observations, explore=False, policy_id=None):
        """Batched inference: a dict of observations (agent / env ids) -> dict of actions,
        or a sequence / stacked array -> array of actions."""
        if isinstance(observations, dict):
            return {k: self.compute_single_action(o, explore, policy_id)
                    for k, o in observations.items()}
        return np.stack([np.asarray(self.compute_single_action(o, explore, policy_id))
                         for o in observations])

    def get_policy(self, policy_id=None):
        """Old-stack view: an object with compute_single_action / compute_actions /
        get_weights / set_weights bound to this algorithm's module ``policy_id``."""
        return _PolicyView(self, policy_id)

    def set_weights(self, weights):
        """Load learner weights (the format ``get_weights`` returns) and sync the
        EnvRunners."""
        self.learner_group.set_weights(weights)
        self._sync_weights(self.get_weights())

    def get_config(self):
        return self.config

    # ---------------------------------------------------------------- module set (multi-agent)
    def add_module(self, module_id, module_spec=None, *, config_overrides=None,
                   new_agent_to_module_mapping_fn=None, new_should_module_be_updated=None,
                   add_to_learners=True, add_to_env_runners=True,
                   add_to_eval_env_runners=True, weights=None):
        """Add an RLModule to a running multi-agent algorithm (reference:
        rllib/algorithms/algorithm.py:2054 add_module): a learner group for it (when it is
        trained), a replay buffer for off-policy algorithms, the module on every EnvRunner
        (inference), the new agent -> module mapping and the trainable set. ``module_spec``:
        an RLModuleSpec (its observation/action spaces; missing ones default to an
        existing module's), or an (observation_space, action_space) tuple. ``weights``:
        initial weights (e.g. a frozen copy of the main policy for league / self-play);
        otherwise the new module keeps its fresh initialisation. Returns the module ids."""
        if not self.is_multi_agent:
            raise ValueError("add_module needs a multi-agent config (config.multi_agent)")
        if module_id in self.module_specs:
            raise ValueError(f"module {module_id!r} already exists")
        ref = next(iter(self.module_specs.values()))
        if isinstance(module_spec, (tuple, list)):
            os_, as_ = module_spec
        else:
            os_ = getattr(module_spec, "observation_space", None) or ref[0]
            as_ = getattr(module_spec, "action_space", None) or ref[1]
        spec = (os_, as_)
        trainable = self._trainable_after(module_id, new_should_module_be_updated)
        self.module_specs = dict(self.module_specs)
        self.module_specs[module_id] = spec
        self.cfg["_module_specs"] = self.module_specs
        if add_to_learners:
            lg = self.learner_group
            # the learners build the module (its network, optimizers and loss) through
            # Learner.add_module on every learner of the group (learner_group.py:494)
            lg.add_module(module_id=module_id, module_spec=spec,
                          config_overrides=config_overrides,
                          new_should_module_be_updated=sorted(trainable, key=str))
            if hasattr(self, "buffers") and module_id in trainable:
                self.buffers[module_id] = self._new_buffer()
            self._set_trainable(trainable)
            if weights is not None:
                lg.set_module_state({module_id: weights})
        w = weights if weights is not None else self.get_weights().get(module_id)
        if new_agent_to_module_mapping_fn is not None:
            self.config.policy_mapping_fn = new_agent_to_module_mapping_fn
            self.cfg["policy_mapping_fn"] = new_agent_to_module_mapping_fn
        if add_to_env_runners:
            self._on_runners(lambda r: r.add_module(module_id, spec, w))
            if new_agent_to_module_mapping_fn is not None:
                fn = new_agent_to_module_mapping_fn
                self._on_runners(lambda r: r.set_mapping_fn(fn))
        if add_to_eval_env_runners and self._eval_runners:
            import cloudpickle

            blob = cloudpickle.dumps(lambda r: r.add_module(module_id, spec, w))
            ray.get([r.apply.remote(blob) for r in self._eval_runners])
        self.weights_version += 1  # runners re-sync every module's weights
        self._sync_weights(self.get_weights())
        return list(self.module_specs)

    def remove_module(self, module_id, *, new_agent_to_module_mapping_fn=None,
                      new_should_module_be_updated=None, remove_from_learners=True,
                      remove_from_env_runners=True, remove_from_eval_env_runners=True):
        """Remove a module (reference: algorithm.py remove_module); the mapping must no
        longer route agents to it."""
        if not self.is_multi_agent or module_id not in self.module_specs:
            raise ValueError(f"unknown module {module_id!r}")
        trainable = self._trainable_after(None, new_should_module_be_updated) - {module_id}
        self.module_specs = {k: v for k, v in self.module_specs.items() if k != module_id}
        self.cfg["_module_specs"] = self.module_specs
        if new_agent_to_module_mapping_fn is not None:
            self.config.policy_mapping_fn = new_agent_to_module_mapping_fn
            self.cfg["policy_mapping_fn"] = new_agent_to_module_mapping_fn
            fn = new_agent_to_module_mapping_fn
            self._on_runners(lambda r: r.set_mapping_fn(fn))
        if remove_from_env_runners:
            self._on_runners(lambda r: r.remove_module(module_id))
        if remove_from_eval_env_runners and self._eval_runners:
            import cloudpickle

            blob = cloudpickle.dumps(lambda r: r.remove_module(module_id))
            ray.get([r.apply.remote(blob) for r in self._eval_runners])
        if remove_from_learners:
            lg = self.learner_group
            lg.remove_module(module_id)
            if hasattr(self, "buffers"):
                self.buffers.pop(module_id, None)
        self._set_trainable(trainable)
        return list(self.module_specs)

    def add_policy(self, policy_id, policy_cls=None, policy=None, *, observation_space=None,
                   action_space=None, config=None, policy_state=None,
                   policy_mapping_fn=None, policies_to_train=None, **kwargs):
        """Old-stack spelling of ``add_module`` (reference: algorithm.py:1929)."""
        ref = next(iter(self.module_specs.values())) if self.is_multi_agent else None
        spaces = (observation_space or (ref[0] if ref else self.observation_space),
                  action_space or (ref[1] if ref else self.action_space))
        weights = policy_state.get("weights", policy_state) if isinstance(policy_state, dict) \
            else None
        self.add_module(policy_id, spaces, new_agent_to_module_mapping_fn=policy_mapping_fn,
                        new_should_module_be_updated=policies_to_train, weights=weights)
        return self.get_policy(policy_id)

    def remove_policy(self, policy_id, *, policy_mapping_fn=None, policies_to_train=None,
                      **kwargs):
        self.remove_module(policy_id, new_agent_to_module_mapping_fn=policy_mapping_fn,
                           new_should_module_be_updated=policies_to_train)

    def _trainable_after(self, new_id, spec):
        """The trainable module set after add/remove: ``spec`` is a list / set of ids or a
        callable(module_id) -> bool; None keeps the current set (+ the new module)."""
        lg = getattr(self, "learner_group", None)
        cur = set(getattr(lg, "trainable", ()) or self.module_specs)
        ids = set(self.module_specs) | ({new_id} if new_id is not None else set())
        if spec is None:
            return cur | ({new_id} if new_id is not None else set())
        if callable(spec):
            return {m for m in ids if spec(m)}
        return set(spec)

    def _set_trainable(self, trainable):
        lg = getattr(self, "learner_group", None)
        if lg is not None and hasattr(lg, "trainable"):
            lg.trainable = set(trainable)
        self.config.policies_to_train = sorted(trainable, key=str)

    def _on_runners(self, fn):
        """fn(runner) on the local runner and every remote EnvRunner (through apply)."""
        import cloudpickle

        if self._runners.num_actors():
            blob = cloudpickle.dumps(fn)
            self._foreach_runner(lambda r: r.apply.remote(blob))
        if self.local_runner is not None:
            fn(self.local_runner)

    @property
    def env_runner_group(self):
        return _EnvRunnerGroupView(self)

    workers = env_runner_group

    def export_policy_model(self, export_dir: str, policy_id=None, onnx=None):
        """Save the inference module: ``model.pt`` (a TorchScript trace when the module
        traces, else the pickled module) plus ``state_dict.pt``."""
        import torch

        if onnx:
            raise NotImplementedError("ONNX export needs the onnx package (not installed)")
        os.makedirs(export_dir, exist_ok=True)
        m = self.get_module(policy_id)
        torch.save(m.state_dict(), os.path.join(export_dir, "state_dict.pt"))
        try:
            sample = torch.as_tensor(self.observation_space.sample()[None])
            if self.cfg.get("module_kind", "actor_critic") == "actor_critic":
                traced = torch.jit.trace(lambda x: m.forward_inference(x)[
                    "action_dist_inputs"], sample)
            else:
                traced = torch.jit.trace(m, sample.float())
            traced.save(os.path.join(export_dir, "model.pt"))
        except Exception:  # noqa: BLE001  (untraceable module: pickle it)
            torch.save(m, os.path.join(export_dir, "model.pt"))
        return export_dir

    export_model = export_policy_model

    def save_checkpoint(self, checkpoint_dir: str):
        self.save(checkpoint_dir)
        return checkpoint_dir

    def load_checkpoint(self, checkpoint):
        self.restore(checkpoint)

    compute_action = compute_single_action

    # ---------------------------------------------------------------- checkpoints
    def get_weights(self):
        return self.learner_group.get_weights()

    def get_state(self):
        return {"learner": self.learner_group.get_state(), "iteration": self.iteration,
                "total_env_steps": self.total_env_steps, "config": self.cfg,
                "algorithm_class": type(self)}

    @classmethod
    def from_state(cls, state: dict) -> "Algorithm":
        """A new Algorithm from a ``get_state()`` dict (reference: algorithm.py:353): the
        class recorded in the state (or ``cls``), its config rebuilt from the state's
        config, then the learner / counters state loaded."""
        algo_cls = state.get("algorithm_class") or cls
        if not isinstance(algo_cls, type) or not issubclass(algo_cls, Algorithm):
            raise ValueError(f"state names no Algorithm class ({algo_cls!r})")
        from ray_amd.rllib.algorithms.registry import get_config_class

        cfg_state = {k: v for k, v in dict(state["config"]).items()
                     if not k.startswith("_") and k not in ("module_kind",)}
        config = get_config_class(algo_cls)().update_from_dict(cfg_state)
        algo = algo_cls(config)
        algo.set_state(state)
        return algo

    def restore_workers(self, workers=None):
        """Old-stack name (reference: algorithm.py:1429): probe the given (default: all)
        EnvRunners, recreate the dead ones and push the current weights to them."""
        restored = self.restore_env_runners()
        if restored:
            self._sync_weights(self.get_weights())
        return restored

    @staticmethod
    def validate_env(env, env_context) -> None:
        """Hook to validate a freshly created env (reference: algorithm.py:2680; the
        default accepts every env). Subclasses override it to reject envs they cannot
        train on; it runs on every env an EnvRunner of this algorithm creates."""
        return None

    def set_state(self, s):
        self.learner_group.set_state(s["learner"])
        self.iteration = s["iteration"]
        self.total_env_steps = s["total_env_steps"]
        self._sync_weights(self.get_weights())

    def save(self, checkpoint_dir: str | None = None):
        import tempfile

        d = checkpoint_dir or tempfile.mkdtemp(prefix="rllib_ckpt_")
        os.makedirs(d, exist_ok=True)
        import cloudpickle  # policy_mapping_fn is usually a lambda

        with open(os.path.join(d, "algorithm_state.pkl"), "wb") as f:
            cloudpickle.dump(self.get_state(), f)
        from ray_amd.train._checkpoint import Checkpoint

        return Checkpoint(d)

    save_to_path = save

    def restore(self, checkpoint):
        path = checkpoint.path if hasattr(checkpoint, "path") else checkpoint
        with open(os.path.join(path, "algorithm_state.pkl"), "rb") as f:
            self.set_state(pickle.load(f))
        self.callbacks.on_checkpoint_loaded(algorithm=self)

    restore_from_path = restore

    @classmethod
    def from_checkpoint(cls, checkpoint, config=None):
        path = checkpoint.path if hasattr(checkpoint, "path") else checkpoint
        with open(os.path.join(path, "algorithm_state.pkl"), "rb") as f:
            state = pickle.load(f)
        if config is None:
            from ray_amd.rllib.algorithms.registry import get_config_class

            config = get_config_class(cls)().update_from_dict(state["config"])
        algo = cls(config)
        algo.set_state(state)
        return algo

    def stop(self):
        self._runners.clear()
        if self._policy_server is not None:
            try:
                ray.kill(self._policy_server)
            except Exception:  # noqa: BLE001
                pass
            self._policy_server = None
        if getattr(self, "_policy_server_local", None) is not None:
            self._policy_server_local.shutdown()
            self._policy_server_local = None
        for r in self._eval_runners:
            try:
                ray.kill(r)
            except Exception:  # noqa: BLE001
                pass
        self._eval_runners = []
        self.learner_group.shutdown()

    def __del__(self):
        pass


from ray_amd.rllib.policy import Policy as _Policy  # noqa: E402


class _PolicyView(_Policy):
    def __init__(self, algo, policy_id):
        self.algo, self.policy_id = algo, policy_id
        self.observation_space = algo.observation_space
        self.action_space = algo.action_space
        self.config = {}
        self.global_timestep = 0

    @property
    def model(self):
        return self.algo.get_module(self.policy_id)

    def compute_single_action(self, obs, state=None, explore=None, **kw):
        a = self.algo.compute_single_action(obs, bool(explore), self.policy_id)
        return a, [], {}

    def compute_actions(self, obs_batch, state_batches=None, explore=None, **kw):
        return self.algo.compute_actions(obs_batch, bool(explore), self.policy_id), [], {}

    def compute_log_likelihoods(self, actions, obs_batch, **kw):
        """log pi(a | s) of the module's current weights (reference: Policy.
        compute_log_likelihoods): categorical for discrete actions, the diagonal Gaussian
        (or SAC's squashed Gaussian) for Box actions, greedy one-hot for Q modules."""
        import torch

        m = self.algo.get_module(self.policy_id)
        obs = np.asarray(obs_batch, np.float32)
        f = getattr(self.algo, "_infer_filter", None)
        x = torch.as_tensor(obs)
        if f is not None:
            x = f.normalize(x)
        a = torch.as_tensor(np.asarray(actions))
        kind = self.algo.cfg.get("module_kind", "actor_critic")
        with torch.no_grad():
            if kind == "q":
                greedy = m(x.float()).argmax(-1)
                return np.where(greedy.numpy() == a.numpy(), 0.0, -np.inf)
            if kind == "sac":
                return m.logp_of(x.float(), a.float()).double().numpy()
            di = m.forward_inference(x)["action_dist_inputs"].float()
            if hasattr(self.action_space, "n"):
                return torch.log_softmax(di, -1).gather(-1, a.long()[:, None])[:, 0] \
                    .double().numpy()
            from ray_amd.rllib.core.rl_module.default import gaussian_logp

            mean, log_std = di.chunk(2, -1)
            return gaussian_logp(a.float(), mean, log_std).double().numpy()

    def get_weights(self):
        w = self.algo.get_weights()
        return w[self.policy_id] if self.policy_id is not None and self.policy_id in w else w

    def set_weights(self, weights):
        if self.policy_id is not None and self.algo.is_multi_agent:
            full = dict(self.algo.get_weights())
            full[self.policy_id] = weights
            weights = full
        self.algo.set_weights(weights)


class _EnvRunnerGroupView:
    """``algo.env_runner_group`` / ``algo.workers``: the EnvRunner actors (or the local
    runner when there are none)."""

    def __init__(self, algo):
        self.algo = algo

    def _all(self):
        return list(self.algo.env_runners) or [self.algo.local_runner]

    def foreach_env_runner(self, func, local_env_runner=True, remote_worker_ids=None):
        import cloudpickle

        out = []
        if self.algo.env_runners:
            blob = cloudpickle.dumps(func)
            runners = self.algo.env_runners
            if remote_worker_ids is not None:
                runners = [runners[i - 1] for i in remote_worker_ids]
            out = ray.get([r.apply.remote(blob) for r in runners])
        elif local_env_runner:
            out = [func(self.algo.local_runner)]
        return out

    foreach_worker = foreach_env_runner

    def num_healthy_remote_workers(self) -> int:
        return self.algo._runners.num_healthy_actors()

    def probe_unhealthy_env_runners(self):
        return self.algo.restore_env_runners()

    probe_unhealthy_workers = probe_unhealthy_env_runners

    num_healthy_remote_env_runners = num_healthy_remote_workers
    num_remote_workers = num_healthy_remote_workers

    def sync_weights(self, *a, **k):
        self.algo._sync_weights(self.algo.get_weights())

    def local_env_runner(self):
        return self.algo.local_runner

