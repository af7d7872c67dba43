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
        self.learners = {mid: make(os_, as_) for mid, (os_, as_) in specs.items()}
        self.trainable = set(trainable) if trainable else set(specs)

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
        if nr > 0:
            self.env_runners = [runner_cls.options(**opts).remote(self.cfg, i + 1)
                                for i in range(nr)]
            ray.get([r.ping.remote() for r in self.env_runners])
            self.local_runner = None
        else:
            self.env_runners = []
            self.local_runner = local_cls(self.cfg, 0)
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

    # ---------------------------------------------------------------- weights
    def _sync_weights(self, weights):
        self.weights_version += 1
        if self.env_runners:
            ref = ray.put(weights)
            ray.get([r.set_weights.remote(ref, self.weights_version) for r in self.env_runners])
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
        elif self.env_runners:
            ms = ray.get([r.get_metrics.remote() for r in self.env_runners])
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
        if self.config.evaluation_interval and self.iteration % self.config.evaluation_interval \
                == 0:
            self.callbacks.on_evaluate_start(algorithm=self, metrics_logger=self.metrics)
            out["evaluation"] = self.evaluate()
            self.callbacks.on_evaluate_end(algorithm=self, evaluation_metrics=out["evaluation"],
                                           metrics_logger=self.metrics)
        self.callbacks.on_train_result(algorithm=self, result=out, metrics_logger=self.metrics)
        extra = self.metrics.reduce_all()
        if extra:
            out.setdefault("custom_metrics", {}).update(extra)
        return out

    def training_step(self) -> dict:
        raise NotImplementedError

    def _sample(self, total: int):
        """Synchronous parallel sampling of >= total env steps (reference:
        rllib/execution/rollout_ops.py:synchronous_parallel_sample)."""
        cfg = self.config
        per = cfg.rollout_fragment_length
        batches = []
        got = 0
        while got < total:
            if self.env_runners:
                bs = ray.get([r.sample.remote(per) for r in self.env_runners])
            else:
                bs = [self.local_runner.sample(per)]
            for b in bs:
                got += b["env_steps"]
            batches.extend(bs)
        self.total_env_steps += got
        return batches

    def evaluate(self) -> dict:
        runner = self._runner_cls(self.cfg, 999)
        runner.set_weights(self.get_weights(), None)
        n = self.config.evaluation_duration
        rets = []
        while len(rets) < n:
            runner.sample(self.config.rollout_fragment_length, explore=False)
            rets.extend(runner.get_metrics()["episode_returns"])
        return {"env_runners": {"episode_return_mean": float(np.mean(rets[:n]))}}

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
                "total_env_steps": self.total_env_steps, "config": self.cfg}

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
        for r in self.env_runners:
            try:
                ray.kill(r)
            except Exception:
                pass
        self.env_runners = []
        self.learner_group.shutdown()

    def __del__(self):
        pass


class _PolicyView:
    def __init__(self, algo, policy_id):
        self.algo, self.policy_id = algo, policy_id
        self.observation_space = algo.observation_space
        self.action_space = algo.action_space

    @property
    def model(self):
        return self.algo.get_module(self.policy_id)

    def compute_single_action(self, obs, state=None, explore=None, **kw):
        a = self.algo.compute_single_action(obs, bool(explore), self.policy_id)
        return a, [], {}

    def compute_actions(self, obs_batch, state_batches=None, explore=None, **kw):
        return self.algo.compute_actions(obs_batch, bool(explore), self.policy_id), [], {}

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
        return len(self.algo.env_runners)

    num_healthy_remote_env_runners = num_healthy_remote_workers
    num_remote_workers = num_healthy_remote_workers

    def sync_weights(self, *a, **k):
        self.algo._sync_weights(self.algo.get_weights())

    def local_env_runner(self):
        return self.algo.local_runner

