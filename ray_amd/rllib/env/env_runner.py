"""Single-agent EnvRunner (reference: rllib/env/single_agent_env_runner.py,
rllib/evaluation/rollout_worker.py).

Each runner steps ``num_envs_per_env_runner`` envs in lock-step (vectorised)
and returns time-major [T, B] fragments as numpy arrays; the fragment travels
to the learner through the shared-memory object store (zero-copy), where GAE /
V-trace run as HIP kernels. Episodes auto-reset; ``terminateds`` marks episode
ends (truncation is folded into termination: no bootstrap across a time-limit
cut)."""

from __future__ import annotations

import os
import time

import numpy as np
import torch

from ray_amd.rllib.env.envs import make_env


def _grow(x, n):
    """Append n uninitialised-but-zeroed rows along the time axis."""
    if x is None:
        return None
    return np.concatenate([x, np.zeros((n,) + x.shape[1:], x.dtype)], 0)


class SingleAgentEnvRunner:
    def __init__(self, config: dict, worker_index: int = 0):
        torch.set_num_threads(int(config.get("num_cpus_per_env_runner", 1) or 1))
        self.config = config
        self.worker_index = worker_index
        n = int(config.get("num_envs_per_env_runner", 1))
        seed = config.get("seed")
        from ray_amd.rllib.env.vector_env import VectorEnv

        self.envs = []
        from ray_amd.rllib.env.env_context import EnvContext

        env_spec = config["env"]
        if env_spec is None and callable(config.get("input_")):
            # no local env: the input factory provides an ExternalEnv (PolicyServerInput:
            # remote simulators drive the episodes; reference: offline_data(input_=...))
            from ray_amd.rllib.offline.io_context import IOContext

            inp = config["input_"]
            env_spec = (lambda ec, inp=inp: inp(IOContext(config=config,
                                                          worker_index=ec.worker_index)))
        for i in range(n):
            ec = EnvContext(config.get("env_config") or {}, worker_index=worker_index,
                            vector_index=i, remote=worker_index > 0,
                            num_workers=config.get("num_env_runners"))
            ec.setdefault("seed", (seed or 0) * 1000 + worker_index * 100 + i)
            e = make_env(env_spec, ec)
            if config.get("_validate_env") is not None:  # Algorithm.validate_env
                config["_validate_env"](e, ec)
            if isinstance(e, VectorEnv):  # its sub-environments join the lock-step batch
                subs = e.get_sub_environments()
                if not subs:
                    raise ValueError(f"{type(e).__name__} exposes no sub-environments; "
                                     "EnvRunners step concrete envs")
                self.envs.extend(subs)
            else:
                self.envs.append(e)
        n = len(self.envs)
        self.observation_space = self.envs[0].observation_space
        self.action_space = self.envs[0].action_space
        # ConnectorV2 pipelines: env -> module (per batched step) and module -> env
        from ray_amd.rllib.callbacks import EpisodeState, MetricsLogger, make_callbacks
        from ray_amd.rllib.connectors.connector_v2 import build_pipeline

        self.env_to_module = build_pipeline(config.get("env_to_module_connector"),
                                            self.observation_space, self.action_space)
        if config.get("observation_filter") == "MeanStdFilter" and \
                not any(getattr(c, "learner_side", False) for c in self.env_to_module.connectors):
            from ray_amd.rllib.connectors.env_to_module import MeanStdFilter

            self.env_to_module.append(MeanStdFilter(self.observation_space, self.action_space))
        # learner-side connectors (MeanStdFilter: stats owned by the learner) run last and
        # are NOT applied to the recorded observations
        self._pre = [c for c in self.env_to_module.connectors
                     if not getattr(c, "learner_side", False)]
        self._post = [c for c in self.env_to_module.connectors
                      if getattr(c, "learner_side", False)]
        self.module_to_env = build_pipeline(config.get("module_to_env_connector"),
                                            self.observation_space, self.action_space)
        # AlgorithmConfig env / rollout semantics (reference: algorithm_config.py:1385-1398
        # clip_rewards, normalize_actions, clip_actions; :1515 batch_mode)
        self.clip_rewards = config.get("clip_rewards")
        self.batch_mode = config.get("batch_mode") or "truncate_episodes"
        if self.batch_mode not in ("truncate_episodes", "complete_episodes"):
            raise ValueError(f"batch_mode must be 'truncate_episodes' or 'complete_episodes', "
                             f"got {self.batch_mode!r}")
        kind = config.get("module_kind", "actor_critic")
        self._final_clip = False
        if hasattr(self.action_space, "low"):
            from ray_amd.rllib.connectors.module_to_env import (ClipActions,
                                                                NormalizeAndClipActions)

            have = {type(c) for c in self.module_to_env.connectors}
            if kind == "sac":
                # the SAC actor already rescales its tanh output to the Box bounds
                self._final_clip = True
            elif config.get("normalize_actions", True):
                # the policy acts in [-1, 1]; unsquash to the bounds (and clip) for env.step
                if NormalizeAndClipActions not in have:
                    self.module_to_env.append(NormalizeAndClipActions(self.observation_space,
                                                                      self.action_space))
            elif config.get("clip_actions", False) and ClipActions not in have:
                self.module_to_env.append(ClipActions(self.observation_space,
                                                      self.action_space))
        self.module_obs_space = self.env_to_module.observation_space
        self.callbacks = make_callbacks(config.get("callbacks_class"))
        self.metrics = MetricsLogger()
        for e in self.envs:
            self.callbacks.on_environment_created(env_runner=self, env=e,
                                                  env_context=config.get("env_config"),
                                                  metrics_logger=self.metrics)
        act_dummy = 0 if hasattr(self.action_space, "n") else \
            np.zeros(self.action_space.shape, np.float32)
        self._act_dummy = act_dummy
        self.episodes = [EpisodeState(i, worker_index, act_dummy) for i in range(n)]
        self._next_eid = n
        from ray_amd.rllib.core.rl_module import RLModule

        self.module_kind = config.get("module_kind", "actor_critic")
        if self.module_kind == "q":
            from ray_amd.rllib.core.rl_module import QModule

            mc = dict(config.get("model") or {})
            mc["dueling"] = config.get("dueling", True)
            self.module = QModule(self.module_obs_space, self.action_space, mc)
        elif self.module_kind == "sac":
            from ray_amd.rllib.core.rl_module import SquashedGaussianPolicy

            self.module = SquashedGaussianPolicy(self.module_obs_space, self.action_space,
                                                 config.get("policy_model_config") or
                                                 config.get("model"))
        else:
            from ray_amd.rllib.core.rl_module.rl_module import build_module

            self.module = build_module(config, self.module_obs_space, self.action_space)
        self.module.eval()
        # stateful (recurrent) modules: one state per env, carried across fragments, zeroed
        # at episode starts; each fragment records the state it started from
        self._stateful = bool(getattr(self.module, "is_stateful", lambda: False)()) and \
            self.module_kind not in ("q", "sac")
        if self._stateful:
            init = self.module.get_initial_state()
            self._state = {k: np.repeat(np.asarray(v, np.float32)[None], n, 0)
                           for k, v in init.items()}
            self._state0 = {k: np.asarray(v, np.float32) for k, v in init.items()}
        ac_module = self.module_kind in ("actor_critic", "pg")  # PPO / IMPALA / APPO / A2C
        self.device = torch.device("cpu")
        if config.get("num_gpus_per_env_runner") and worker_index > 0 and \
                not torch.cuda.is_initialized():
            # a runner process drives one stream: cap its HIP hardware queues before the
            # runtime starts (8 runners x 8 queues beside the learner oversubscribe the
            # queue slots, and oversubscribed queues are time-sliced)
            os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RAY_AMD_RUNNER_HW_QUEUES", "1")
        if config.get("num_gpus_per_env_runner") and torch.cuda.is_available():
            self.device = torch.device("cuda", 0)
            self.module.to(self.device)
            if ac_module and getattr(self.module, "is_image", False):
                # bf16 channels-last weights: the conv encoder runs on the MFMA kernels and
                # reads the uint8 frames directly (weights arrive fp32, cast on load)
                self.module.to(torch.bfloat16).to(memory_format=torch.channels_last)
        # CPU conv policies keep bf16 weights (AVX-512 BF16 convolutions and half the FC
        # weight bytes per step), matching the learner's bf16 compute. Measured per 5-frame
        # Nature-CNN step on the MI355X host (EPYC 9575F, scripts/cpu_infer_bf16_bench.py):
        # fp32 0.68 ms, bf16 autocast 0.52 ms, bf16 weights 0.39 ms. fp32 with
        # env_runner_bf16=False. Synced fp32 weights are cast on load (load_state_dict).
        self._cpu_bf16 = (self.device.type == "cpu" and ac_module
                          and getattr(self.module, "is_image", False)
                          and config.get("env_runner_bf16", config.get("learner_bf16", True)))
        if self._cpu_bf16:
            self.module.to(torch.bfloat16).to(memory_format=torch.channels_last)
        # GPU discrete policies: the whole inference step as one HIP graph (gpu_policy.py)
        self._graphed = (self.device.type == "cuda" and ac_module
                         and not self._stateful and hasattr(self.action_space, "n")
                         and os.environ.get("RAY_AMD_RUNNER_GRAPH", "1") == "1")
        self._gpol = None
        # the runners' shared GPU inference process (num_gpus_per_policy_server)
        self._pclient = None
        srv = config.get("_policy_server")
        if srv is not None and worker_index > 0 and ac_module and not self._stateful:
            from ray_amd.rllib.env.policy_server import PolicyClient

            path, n_slots, pB, oshape, na = srv
            self._pclient = PolicyClient(path, worker_index - 1, n_slots, pB, oshape, na)
            self._graphed = True
        self._act_rng = np.random.default_rng(
            None if seed is None else seed * 7919 + worker_index)
        self.obs = []
        for i, e in enumerate(self.envs):
            o, _ = e.reset(seed=None if seed is None else seed * 1000 + worker_index * 100 + i)
            self.obs.append(o)
            self.episodes[i].id_ = i
            self.callbacks.on_episode_start(episode=self.episodes[i], env_runner=self,
                                            env_index=i, metrics_logger=self.metrics)
        self.ep_ret = np.zeros(n)
        self.ep_len = np.zeros(n, dtype=np.int64)
        self.done_returns = []
        self.done_lengths = []
        self.weights_version = -1
        self.total_steps = 0
        self.epsilon = 1.0
        # SingleAgentEpisode recording (episode replay buffers / sample_episodes)
        self._record = bool(config.get("_record_episodes"))
        self._eps = None

    # ---------------------------------------------------------------- weights
    def set_weights(self, weights, version: int = 0):
        if version is not None and version == self.weights_version:
            return
        weights = dict(weights)
        cstate = weights.pop("__connector_state__", None)
        if cstate is not None:  # learner-owned filter statistics
            for c in self._post:
                c.set_state(cstate)
        sd = {k: (v if isinstance(v, torch.Tensor) else torch.as_tensor(v))
              for k, v in weights.items()}
        self.module.load_state_dict(sd)
        self.weights_version = version

    def get_weights(self):
        # fp32 out (the runner may hold bf16 inference weights)
        return {k: (v.detach().cpu().float() if v.is_floating_point() else v.detach().cpu())
                for k, v in self.module.state_dict().items()}

    def apply(self, fn_blob):
        """Run ``fn(env_runner)`` here (Algorithm.env_runner_group.foreach_env_runner)."""
        import cloudpickle

        return cloudpickle.loads(fn_blob)(self)

    def ping(self):
        return self.worker_index

    # ---------------------------------------------------------------- sampling
    def sample_episodes(self, num_timesteps: int | None = None, explore: bool = True,
                        epsilon: float | None = None):
        """Sample and return the SingleAgentEpisode chunks of the rollout (finished
        episodes, then the ongoing chunks, which continue in the next call; reference:
        SingleAgentEnvRunner.sample returning episodes)."""
        rec = self._record
        self._record = True
        try:
            return self.sample(num_timesteps, explore, epsilon)["episodes"]
        finally:
            self._record = rec

    def sample(self, num_timesteps: int | None = None, explore: bool = True,
               epsilon: float | None = None, with_metrics: bool = False):
        T = int(num_timesteps or self.config.get("rollout_fragment_length", 50))
        B = len(self.envs)
        if self._record and self._eps is None:
            from ray_amd.rllib.env.single_agent_episode import SingleAgentEpisode

            self._eps = [SingleAgentEpisode(observation_space=self.module_obs_space,
                                            action_space=self.action_space) for _ in range(B)]
        done_eps = []
        osh = self.observation_space.shape
        obs_buf = np.empty((T, B) + tuple(osh), dtype=self.observation_space.dtype) \
            if not self._pre else None  # connector output shape known after step 0
        discrete = hasattr(self.action_space, "n")
        act_buf = np.empty((T, B) if discrete else (T, B) + tuple(self.action_space.shape),
                           dtype=np.int64 if discrete else np.float32)
        rew = np.zeros((T, B), np.float32)
        term = np.zeros((T, B), np.float32)
        trunc = np.zeros((T, B), np.float32)
        logp = np.zeros((T, B), np.float32)
        dist_in = None
        next_obs_buf = None
        if self.module_kind in ("q", "sac"):
            next_obs_buf = np.empty_like(obs_buf)
        resets = None
        if self._stateful:
            state_in = {k: v.copy() for k, v in self._state.items()}
            resets = np.zeros((T, B), np.float32)
        t0 = time.perf_counter()
        # batch_mode "complete_episodes": every env runs its episode to the end once it has
        # stepped T times, then idles (padding rows: loss_mask 0, terminated); the fragment
        # is [T' >= T, B] and every env starts the next call at a fresh episode
        complete = self.batch_mode == "complete_episodes"
        active = np.ones(B, bool)
        env_steps = np.zeros(B, np.int64)
        mask = np.ones((T, B), np.float32) if complete else None
        reset_next = np.zeros(B, bool)
        cap = T
        t = 0
        while (t < T) if not complete else active.any():
            rec, ob = self._module_obs(np.stack(self.obs), explore)
            if obs_buf is None:
                obs_buf = np.empty((cap,) + rec.shape, dtype=rec.dtype)
                if next_obs_buf is not None:
                    next_obs_buf = np.empty_like(obs_buf)
            if t >= cap:  # complete_episodes ran past T: grow every time-major buffer
                grow = cap
                obs_buf, act_buf, rew, term, trunc, logp, mask = (
                    _grow(x, grow) for x in (obs_buf, act_buf, rew, term, trunc, logp, mask))
                if next_obs_buf is not None:
                    next_obs_buf = _grow(next_obs_buf, grow)
                if dist_in is not None:
                    dist_in = _grow(dist_in, grow)
                if resets is not None:
                    resets = _grow(resets, grow)
                cap += grow
            obs_buf[t] = rec
            if resets is not None and reset_next.any():  # episode starts in this row
                resets[t, reset_next] = 1.0
                reset_next[:] = False
            if self._record:
                for i in range(B):
                    if not self._eps[i].observations:
                        self._eps[i].add_env_reset(rec[i])
            with torch.no_grad():
                x = None if (self._graphed and not self._stateful) else \
                    torch.from_numpy(np.ascontiguousarray(ob)).to(self.device)
                if self.module_kind == "q":
                    q = self.module(x)
                    a = q.argmax(-1).cpu().numpy()
                    eps = self.epsilon if epsilon is None else epsilon
                    if explore:
                        rnd = np.random.random(B) < eps
                        a = np.where(rnd, np.random.randint(0, self.action_space.n, B), a)
                    lp = np.zeros(B, np.float32)
                elif self.module_kind == "sac":
                    at, lpt = self.module(x, explore)
                    a = at.float().cpu().numpy()
                    lp = lpt.float().cpu().numpy()
                else:
                    if self._stateful:
                        st = {k: torch.from_numpy(v).to(self.device)
                              for k, v in self._state.items()}
                        out = self.module.forward_inference(x, state=st)
                        self._state = {k: v.float().cpu().numpy()
                                       for k, v in out["state_out"].items()}
                    elif self._graphed:
                        out = None
                    else:
                        out = self.module.forward_inference(x)
                    if out is None:
                        if self._pclient is not None:
                            pol = self._pclient
                        else:
                            if self._gpol is None or self._gpol.obs_shape != ob.shape:
                                from ray_amd.rllib.env.gpu_policy import GraphedDiscretePolicy

                                self._gpol = GraphedDiscretePolicy(
                                    self.module, ob, self.action_space.n, self.device)
                            pol = self._gpol
                        a, lp, d = pol.step(ob, explore, self._act_rng)
                        if dist_in is None:
                            dist_in = np.zeros((cap, B, d.shape[-1]), np.float32)
                        dist_in[t] = d
                        lp = lp.copy()
                    else:
                        di = out["action_dist_inputs"].float()
                        at, lpt = self.module.sample_actions(di, explore)
                        if dist_in is None:
                            dist_in = np.zeros((cap, B, di.shape[-1]), np.float32)
                        if discrete and di.is_cuda:  # one device->host copy per step
                            h = torch.cat([at.float()[:, None], lpt[:, None], di],
                                          1).cpu().numpy()
                            a = h[:, 0].astype(np.int64)
                            lp = h[:, 1]
                            dist_in[t] = h[:, 2:]
                        else:
                            a = at.cpu().numpy()
                            lp = lpt.cpu().numpy()
                            dist_in[t] = di.cpu().numpy()
            act_buf[t] = a
            logp[t] = lp
            a_env = a
            if len(self.module_to_env):
                a_env = self.module_to_env(rl_module=self.module,
                                           batch={"actions": a, "actions_for_env": a},
                                           episodes=self.episodes,
                                           explore=explore)["actions_for_env"]
            for i, env in enumerate(self.envs):
                if complete and not active[i]:  # padding row of an env that is done
                    rew[t, i] = 0.0
                    term[t, i] = 1.0
                    trunc[t, i] = 0.0
                    mask[t, i] = 0.0
                    if next_obs_buf is not None:
                        next_obs_buf[t, i] = obs_buf[t, i]
                    if self._stateful:  # it starts the next call from the initial state
                        for k, v in self._state0.items():
                            self._state[k][i] = v
                    continue
                ai = a_env[i]
                if not discrete and self._final_clip:
                    ai = np.clip(ai, self.action_space.low, self.action_space.high)
                o, r, te, tr, _ = env.step(ai if not discrete else int(ai))
                env_steps[i] += 1
                if complete:
                    mask[t, i] = 1.0
                rt = self._clip_reward(r)  # the train batch's reward; metrics keep r
                rew[t, i] = rt
                self.ep_ret[i] += r
                self.ep_len[i] += 1
                ep = self.episodes[i]
                ep.t += 1
                ep.total_reward += float(r)
                ep.prev_action = a[i]
                ep.prev_reward = float(r)
                self.callbacks.on_episode_step(episode=ep, env_runner=self, env_index=i,
                                               metrics_logger=self.metrics)
                if next_obs_buf is not None:
                    next_obs_buf[t, i] = self._module_obs(o[None], explore, update=False)[0][0] \
                        if self._pre else o
                if self._record:
                    nxt = next_obs_buf[t, i] if next_obs_buf is not None else (
                        self._module_obs(o[None], explore, update=False)[0][0] if self._pre
                        else o)
                    self._eps[i].add_env_step(np.array(nxt), a[i], rt, terminated=bool(te),
                                              truncated=bool(tr) and not te)
                    if te or tr:
                        from ray_amd.rllib.env.single_agent_episode import SingleAgentEpisode

                        done_eps.append(self._eps[i])
                        self._eps[i] = SingleAgentEpisode(
                            observation_space=self.module_obs_space,
                            action_space=self.action_space)
                if te or tr:
                    term[t, i] = 1.0 if (te or not self.config.get("bootstrap_truncated")) \
                        else 0.0
                    trunc[t, i] = float(tr)
                    self.done_returns.append(float(self.ep_ret[i]))
                    self.done_lengths.append(int(self.ep_len[i]))
                    self.ep_ret[i] = 0.0
                    self.ep_len[i] = 0
                    self.callbacks.on_episode_end(episode=ep, env_runner=self, env_index=i,
                                                  metrics_logger=self.metrics)
                    for k, v in ep.custom_metrics.items():
                        self.metrics.log_value(k, v)
                    o, _ = env.reset()
                    if self._stateful:  # the next episode starts from the initial state
                        for k, v in self._state0.items():
                            self._state[k][i] = v
                        reset_next[i] = True
                    ep.reset(self._act_dummy, self._next_eid)
                    self._next_eid += 1
                    self.callbacks.on_episode_start(episode=ep, env_runner=self, env_index=i,
                                                    metrics_logger=self.metrics)
                    if complete and env_steps[i] >= T:
                        active[i] = False
                self.obs[i] = o
            t += 1
        if complete:  # trim to the steps taken
            obs_buf, act_buf, rew, term, trunc, logp, mask = (
                x[:t] for x in (obs_buf, act_buf, rew, term, trunc, logp, mask))
            if next_obs_buf is not None:
                next_obs_buf = next_obs_buf[:t]
            if dist_in is not None:
                dist_in = dist_in[:t]
            if resets is not None:
                resets = resets[:t]
        n_real = int(env_steps.sum())
        self.total_steps += n_real
        boot = np.stack(self.obs)
        if self._pre:
            boot = self._module_obs(boot, explore, update=False)[0]
        batch = {"obs": obs_buf, "actions": act_buf, "rewards": rew, "terminateds": term,
                 "truncateds": trunc, "action_logp": logp,
                 "bootstrap_obs": boot, "env_steps": n_real,
                 "sample_time_s": time.perf_counter() - t0,
                 "weights_version": self.weights_version}
        if dist_in is not None:
            batch["action_dist_inputs"] = dist_in
        if mask is not None:
            batch["loss_mask"] = mask
        if resets is not None:
            for k, v in state_in.items():
                batch[f"state_in_{k}"] = v
            batch["resets"] = resets
        if self._record:
            ongoing = []
            for i, e in enumerate(self._eps):
                if len(e):
                    ongoing.append(e)
                    self._eps[i] = e.cut()
            batch["episodes"] = done_eps + ongoing
        if next_obs_buf is not None:
            batch["next_obs"] = next_obs_buf
        if self.config.get("output"):
            if getattr(self, "_writer", None) is None:
                from ray_amd.rllib.offline import JsonWriter, ParquetWriter

                if self.config.get("output_write_method") == "write_parquet":
                    self._writer = ParquetWriter(
                        self.config["output"], self.worker_index,
                        self.config.get("output_max_rows_per_file") or 100_000)
                else:
                    self._writer = JsonWriter(self.config["output"], self.worker_index)
            if next_obs_buf is None:  # next_obs from the rolled-forward observations
                nxt = np.concatenate([obs_buf[1:], np.stack(self.obs)[None]], 0)[:len(obs_buf)]
                batch = dict(batch, next_obs=nxt)
            self._writer.write(batch)
        self.callbacks.on_sample_end(env_runner=self, samples=batch, metrics_logger=self.metrics)
        if with_metrics:  # async samplers: no separate get_metrics call behind a sample
            batch["_metrics"] = self.get_metrics()
        return batch

    def sample_with_meta(self, num_timesteps: int | None = None, explore: bool = True):
        """(batch, meta) as TWO objects (call with ``.options(num_returns=2)``): a driver
        that only routes the batch to learner actors fetches the small meta (env steps,
        episode metrics) and hands the batch's ObjectRef on untouched (IMPALA / APPO)."""
        b = self.sample(num_timesteps, explore, with_metrics=True)
        meta = {"env_steps": b["env_steps"], "_metrics": b.pop("_metrics"),
                "weights_version": b.get("weights_version")}
        return b, meta

    def _module_obs(self, ob, explore, update=True):
        """(observation to record, module input) for a batched env step: the env-to-module
        connectors run in order; learner-side ones (MeanStdFilter) only shape the module
        input, the recorded observation stays un-normalized for the learner."""
        if not self.env_to_module.connectors:
            return ob, ob
        b = {"obs": ob}
        for c in self._pre:
            b = c(rl_module=self.module, batch=b, episodes=self.episodes, explore=explore)
        rec = b["obs"]
        if self._post:
            b = {"obs": rec}
            for c in self._post:
                b = c(rl_module=self.module, batch=b, episodes=self.episodes, explore=explore)
        return rec, b["obs"]

    def _clip_reward(self, r):
        c = self.clip_rewards
        if c is None or c is False:
            return r
        if c is True:  # the reference: np.sign (Atari-style)
            return float(np.sign(r))
        return float(np.clip(r, -float(c), float(c)))

    def get_metrics(self):
        r, ln = self.done_returns, self.done_lengths
        self.done_returns, self.done_lengths = [], []
        return {"episode_returns": r, "episode_lengths": ln, "num_env_steps": self.total_steps,
                "custom_metrics": self.metrics.reduce_all()}

    def set_epsilon(self, eps):
        self.epsilon = eps

    def flush_output(self):
        w = getattr(self, "_writer", None)
        if w is not None and hasattr(w, "flush"):
            w.flush()

    def stop(self):
        self.flush_output()
        for e in self.envs:
            e.close()
