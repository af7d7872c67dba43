"""Multi-agent EnvRunner (reference: rllib/env/multi_agent_env_runner.py,
rllib/env/multi_agent_episode.py).

Steps ``num_envs_per_env_runner`` MultiAgentEnvs; each acting agent is routed to an
RLModule through ``policy_mapping_fn(agent_id, episode_id)`` (evaluated once per agent per
episode), and all agents that share a module are batched into one forward pass.

The output keeps the time-major [T, B] layout the HIP GAE kernel consumes: every
(env, agent, module) triple seen in the fragment is one column of its module's batch.
Rows where that agent did not act (it finished before ``__all__``, or its env was
between episodes under another mapping) are padding: ``terminateds = 1`` so the GAE
recursion never crosses them, and ``loss_mask = 0`` so the learner drops them before
the SGD epochs -- advantages of the real rows are therefore exact.  Agents must act on
every step while alive (simultaneous-move envs); turn-based envs are rejected."""

from __future__ import annotations

import time
from collections import defaultdict

import numpy as np
import torch

from ray_amd.rllib.core.rl_module import RLModule
from ray_amd.rllib.env.envs import make_env

DEFAULT_MODULE_ID = "default_policy"


def _default_mapping(agent_id, episode=None, **kw):
    return DEFAULT_MODULE_ID


class MultiAgentEnvRunner:
    def __init__(self, config: dict, worker_index: int = 0):
        torch.set_num_threads(int(config.get("num_cpus_per_env_runner", 1) or 1))
        self.config = config
        self.worker_index = worker_index
        n = int(config.get("num_envs_per_env_runner", 1))
        seed = config.get("seed")
        self.envs = []
        for i in range(n):
            ec = dict(config.get("env_config") or {})
            ec.setdefault("seed", (seed or 0) * 1000 + worker_index * 100 + i)
            self.envs.append(make_env(config["env"], ec))
        self.mapping_fn = config.get("policy_mapping_fn") or _default_mapping
        self.specs = config["_module_specs"]
        self.modules = {mid: RLModule(os_, as_, config.get("model")).eval()
                        for mid, (os_, as_) in self.specs.items()}
        self.obs, self.alive, self.agent_module = [], [], []
        self.ep_ret = np.zeros(n)
        self.ep_len = np.zeros(n, dtype=np.int64)
        self.ep_agent_ret = [defaultdict(float) for _ in range(n)]
        self._ep_counter = 0
        self.ep_ids = [None] * n
        for i, e in enumerate(self.envs):
            o, _ = e.reset(seed=None if seed is None else seed * 1000 + worker_index * 100 + i)
            self._start_episode(i, o)
        self.done_returns, self.done_lengths = [], []
        self.done_module_returns = defaultdict(list)
        self.weights_version = -1
        self.total_steps = 0

    def _start_episode(self, i, obs):
        if len(self.obs) <= i:
            self.obs.append(None)
            self.alive.append(None)
            self.agent_module.append(None)
        self._ep_counter += 1
        self.ep_ids[i] = f"{self.worker_index}-{i}-{self._ep_counter}"
        self.obs[i] = dict(obs)
        self.alive[i] = set(obs)
        self.agent_module[i] = {}

    def _module_of(self, i, aid):
        m = self.agent_module[i].get(aid)
        if m is None:
            m = self.mapping_fn(aid, self.ep_ids[i])
            if m not in self.modules:
                raise ValueError(f"policy_mapping_fn mapped agent {aid!r} to unknown module "
                                 f"{m!r}; known: {sorted(self.modules)}")
            self.agent_module[i][aid] = m
        return m

    # ---------------------------------------------------------------- weights
    def set_weights(self, weights, version: int = 0):
        if version is not None and version == self.weights_version:
            return
        for mid, w in weights.items():
            if mid in self.modules:
                self.modules[mid].load_state_dict(
                    {k: (v if isinstance(v, torch.Tensor) else torch.as_tensor(v))
                     for k, v in w.items()})
        self.weights_version = version

    def get_weights(self):
        return {mid: {k: v.detach().cpu() for k, v in m.state_dict().items()}
                for mid, m in self.modules.items()}

    def ping(self):
        return self.worker_index

    # ---------------------------------------------------------------- sampling
    def _new_col(self, T, mid):
        os_, as_ = self.specs[mid]
        discrete = hasattr(as_, "n")
        return {
            "obs": np.zeros((T,) + tuple(os_.shape), dtype=os_.dtype),
            "actions": np.zeros((T,) if discrete else (T,) + tuple(as_.shape),
                                dtype=np.int64 if discrete else np.float32),
            "rewards": np.zeros(T, np.float32),
            "terminateds": np.ones(T, np.float32),   # padding rows cut the GAE recursion
            "truncateds": np.zeros(T, np.float32),
            "action_logp": np.zeros(T, np.float32),
            "action_dist_inputs": None,
            "loss_mask": np.zeros(T, np.float32),
        }

    def sample(self, num_timesteps: int | None = None, explore: bool = True):
        T = int(num_timesteps or self.config.get("rollout_fragment_length", 50))
        cols: dict = {}   # (env, agent, module) -> column
        t0 = time.perf_counter()
        for t in range(T):
            groups = defaultdict(list)
            for i in range(len(self.envs)):
                missing = self.alive[i] - set(self.obs[i])
                if missing:
                    raise NotImplementedError(
                        f"agents {sorted(missing)} are alive but did not receive an observation; "
                        "turn-based multi-agent envs are not supported by this runner")
                for aid in sorted(self.alive[i], key=str):
                    groups[self._module_of(i, aid)].append((i, aid))
            actions = [{} for _ in self.envs]
            acted = {}
            for mid, items in groups.items():
                mod = self.modules[mid]
                x = torch.from_numpy(np.stack([self.obs[i][aid] for i, aid in items]))
                with torch.no_grad():
                    di = mod.forward_inference(x)["action_dist_inputs"]
                    a, lp = mod.sample_actions(di, explore)
                a, lp, di = a.cpu().numpy(), lp.cpu().numpy(), di.float().cpu().numpy()
                as_ = self.specs[mid][1]
                for j, (i, aid) in enumerate(items):
                    col = cols.get((i, aid, mid))
                    if col is None:
                        col = cols[(i, aid, mid)] = self._new_col(T, mid)
                    if col["action_dist_inputs"] is None:
                        col["action_dist_inputs"] = np.zeros((T, di.shape[-1]), np.float32)
                    col["obs"][t] = self.obs[i][aid]
                    col["actions"][t] = a[j]
                    col["action_logp"][t] = lp[j]
                    col["action_dist_inputs"][t] = di[j]
                    col["loss_mask"][t] = 1.0
                    col["terminateds"][t] = 0.0
                    aj = a[j]
                    actions[i][aid] = int(aj) if hasattr(as_, "n") else \
                        np.clip(aj, as_.low, as_.high)
                    acted[(i, aid)] = col
            for i, env in enumerate(self.envs):
                o, r, te, tr, _ = env.step(actions[i])
                all_done = bool(te.get("__all__")) or bool(tr.get("__all__"))
                for aid, rv in r.items():
                    self.ep_ret[i] += rv
                    self.ep_agent_ret[i][aid] += rv
                for aid in actions[i]:
                    col = acted[(i, aid)]
                    col["rewards"][t] = r.get(aid, 0.0)
                    done = bool(te.get(aid)) or bool(tr.get(aid)) or all_done
                    if done:
                        col["terminateds"][t] = 1.0 if (te.get(aid) or te.get("__all__") or
                                                        not self.config.get("bootstrap_truncated")
                                                        ) else 0.0
                        col["truncateds"][t] = float(bool(tr.get(aid) or tr.get("__all__")))
                        self.alive[i].discard(aid)
                self.ep_len[i] += 1
                if all_done or not self.alive[i]:
                    self.done_returns.append(float(self.ep_ret[i]))
                    self.done_lengths.append(int(self.ep_len[i]))
                    for aid, rv in self.ep_agent_ret[i].items():
                        self.done_module_returns[self.agent_module[i].get(aid, "?")].append(rv)
                    self.ep_ret[i], self.ep_len[i] = 0.0, 0
                    self.ep_agent_ret[i] = defaultdict(float)
                    o, _ = env.reset()
                    self._start_episode(i, o)
                else:
                    self.obs[i] = {aid: ob for aid, ob in o.items() if aid in self.alive[i]}
        env_steps = T * len(self.envs)
        self.total_steps += env_steps
        modules = {}
        for mid in self.modules:
            keys = sorted((k for k in cols if k[2] == mid), key=lambda k: (k[0], str(k[1])))
            if not keys:
                continue
            b = {f: np.stack([cols[k][f] for k in keys], axis=1)
                 for f in ("obs", "actions", "rewards", "terminateds", "truncateds",
                           "action_logp", "action_dist_inputs", "loss_mask")}
            os_ = self.specs[mid][0]
            boot = np.zeros((len(keys),) + tuple(os_.shape), dtype=os_.dtype)
            for j, (i, aid, m) in enumerate(keys):
                if aid in self.alive[i] and self.agent_module[i].get(aid) == m:
                    boot[j] = self.obs[i][aid]
            b["bootstrap_obs"] = boot
            b["env_steps"] = env_steps
            b["agent_steps"] = int(b["loss_mask"].sum())
            modules[mid] = b
        return {"modules": modules, "env_steps": env_steps,
                "agent_steps": sum(b["agent_steps"] for b in modules.values()),
                "sample_time_s": time.perf_counter() - t0,
                "weights_version": self.weights_version}

    def get_metrics(self):
        out = {"episode_returns": self.done_returns, "episode_lengths": self.done_lengths,
               "module_episode_returns": dict(self.done_module_returns),
               "num_env_steps": self.total_steps}
        self.done_returns, self.done_lengths = [], []
        self.done_module_returns = defaultdict(list)
        return out

    def stop(self):
        for e in self.envs:
            e.close()
