"""Learners and LearnerGroup (reference: rllib/core/learner/learner.py, learner_group.py,
rllib/algorithms/ppo/torch/ppo_torch_learner.py, rllib/algorithms/impala/torch/
impala_torch_learner.py, rllib/algorithms/appo/torch/appo_torch_learner.py).

MI355X learner hot loop (one GPU per learner):
  rollouts [T, B] → HBM (uint8 frames, pinned async H2D) → value forward (bf16
  autocast, MFMA convs/GEMMs) → GAE or V-trace (HIP reverse-scan kernels) →
  advantage standardisation → minibatch epochs: forward → fused PPO loss+grad
  kernel (one pass computes loss, stats and d/dlogits, d/dV) → backward →
  flat-buffer gradient all-reduce over RCCL (multi-learner) → fused AdamW kernel.
"""

from __future__ import annotations

import os

import numpy as np
import torch

from ray_amd.ops import functional as rf
from ray_amd.rllib.core.columns import Columns
from ray_amd.rllib.core.rl_module import RLModule, gaussian_entropy, gaussian_logp
from ray_amd.rllib.core.rl_module.rl_module import build_module

DEFAULT_MODULE_ID = "default_policy"
# batch fields whose leading axis is the env / sequence axis (everything else is [T, B, ...])
_AXIS0 = ("bootstrap_obs", "state_in_h", "state_in_c", "state_out_h", "state_out_c")


def _to_t(x, device, dtype=None, non_blocking=True):
    if isinstance(x, Fragments):
        x = x.materialize()
    t = torch.from_numpy(np.ascontiguousarray(x)) if isinstance(x, np.ndarray) else x
    if device.type == "cuda" and not t.is_pinned() and t.device.type == "cpu":
        t = t.pin_memory()
    t = t.to(device, non_blocking=non_blocking)
    return t if dtype is None else t.to(dtype)


class Fragments:
    """Runner fragments [T, B_i, ...] of one batch field, concatenated along the env axis
    only when materialised: a GPU learner stages them straight into pinned memory
    (``Learner._h2d``), skipping a full host copy of the frame batch."""

    def __init__(self, parts):
        self.parts = [np.ascontiguousarray(p) for p in parts]
        p0 = self.parts[0]
        self.shape = (p0.shape[0], sum(p.shape[1] for p in self.parts)) + tuple(p0.shape[2:])
        self.dtype = p0.dtype
        self.nbytes = sum(p.nbytes for p in self.parts)

    def materialize(self):
        return np.concatenate(self.parts, axis=1)

    def __array__(self, dtype=None, copy=None):
        a = self.materialize()
        return a if dtype is None else a.astype(dtype)


def pad_fragment(b: dict, T: int) -> dict:
    """A [t, B] runner fragment padded to T rows: padding rows are terminated with
    loss_mask 0 (batch_mode="complete_episodes" fragments have per-runner lengths; the
    learners drop masked rows and GAE / V-trace never cross a terminated row)."""
    t0 = b["rewards"].shape[0]
    if t0 == T and "loss_mask" in b:
        return b
    out = {}
    for k, v in b.items():
        if isinstance(v, np.ndarray) and k not in _AXIS0 and v.ndim >= 2 and v.shape[0] == t0:
            pad = np.repeat(v[-1:], T - t0, 0) if k in ("obs", "next_obs") else \
                np.zeros((T - t0,) + v.shape[1:], v.dtype)
            if k == "terminateds":
                pad[:] = 1
            out[k] = np.concatenate([v, pad], 0) if T > t0 else v
        else:
            out[k] = v
    if "loss_mask" not in b:
        m = np.zeros((T,) + b["rewards"].shape[1:], np.float32)
        m[:t0] = 1.0
        out["loss_mask"] = m
    return out


def concat_batches(batches, lazy=()):
    """Concatenate runner fragments along the env (B) axis (keys in ``lazy`` become
    ``Fragments``); fragments of different lengths are padded (``pad_fragment``)."""
    lens = {b["rewards"].shape[0] for b in batches if isinstance(b.get("rewards"), np.ndarray)}
    if len(lens) > 1 or (len(batches) > 1 and any("loss_mask" in b for b in batches)
                         and not all("loss_mask" in b for b in batches)):
        T = max(lens)
        batches = [pad_fragment(b, T) for b in batches]
    out = {}
    for k in batches[0]:
        v = batches[0][k]
        if isinstance(v, np.ndarray):
            axis = 0 if k in _AXIS0 else 1
            if k in lazy and axis == 1 and len(batches) > 1:
                out[k] = Fragments([b[k] for b in batches])
            else:
                out[k] = np.concatenate([b[k] for b in batches], axis=axis)
        elif isinstance(v, (int, float)):
            out[k] = sum(b[k] for b in batches)
    return out



def _default_device(config) -> torch.device:
    if torch.cuda.is_available() and config.get("num_gpus_per_learner", 1):
        return torch.device("cuda", int(os.environ.get("RAY_AMD_LOCAL_DEVICE", "0")))
    return torch.device("cpu")


class TorchLearner:
    """The learner pipeline every RLlib algorithm trains through (reference:
    rllib/core/learner/learner.py — :455 compute_gradients, :475 postprocess_gradients,
    :585 apply_gradients, :1149 update_from_batch, :1192 update_from_episodes, :1237
    _update, :1498/:1531 save_state/load_state; torch_learner.py).

    One update::

        batch -> _convert_batch -> forward_train -> compute_losses (compute_loss_for_module
        per module) -> compute_gradients (backward; with several learners the gradients
        are averaged over the learner group in ONE flat all-reduce on RCCL / gloo)
        -> postprocess_gradients (default: clipping by ``grad_clip`` / ``grad_clip_by``)
        -> apply_gradients (every registered optimizer steps)
        -> after_gradient_based_update (target networks, schedules)

    ``compute_losses`` may return one loss per REGISTERED OPTIMIZER (e.g. SAC's critic /
    actor / alpha): then each loss is back-propagated into that optimizer's parameters
    only (``backward(inputs=...)``). Subclasses build their networks in ``build_module``
    and their optimizers in ``configure_optimizers_for_module``. Learners of one group
    start from rank 0's parameters (broadcast) and apply identical averaged gradients,
    so their weights stay identical."""

    def __init__(self, config: dict, observation_space, action_space, device=None, rank=0,
                 world=1, module_id=DEFAULT_MODULE_ID):
        self.config = config
        self.observation_space = observation_space
        self.action_space = action_space
        self.device = device if device is not None else _default_device(config)
        self.rank, self.world = rank, world
        self.module_id = module_id
        torch.manual_seed(config.get("seed") or 0)
        self._optimizers = {}  # (module_id, name) -> (torch optimizer, params)
        self.metrics = {}
        self.updates = 0
        self.build()
        if self.world > 1:
            self._broadcast_params()

    @property
    def cfg(self) -> dict:
        return self.config

    # ---------------------------------------------------------------- build
    def build(self):
        self.module = self.build_module().to(self.device)
        self.configure_optimizers()

    def build_module(self) -> torch.nn.Module:
        from ray_amd.rllib.core.rl_module.rl_module import build_module

        return build_module(self.config, self.observation_space, self.action_space,
                            self.module_id if self.config.get("is_multi_agent") else None)

    def configure_optimizers(self):
        self.configure_optimizers_for_module(self.module_id, self.config)

    def configure_optimizers_for_module(self, module_id, config):
        """Default: one Adam over the module's trainable parameters at ``lr``."""
        params = [p for p in self.module.parameters() if p.requires_grad]
        self.register_optimizer(module_id=module_id, optimizer=torch.optim.Adam(
            params, lr=config.get("lr") or 1e-3), params=params)

    def register_optimizer(self, *, module_id=DEFAULT_MODULE_ID, optimizer_name="default",
                           optimizer, params=None, lr_or_lr_schedule=None):
        params = list(params) if params is not None else \
            [p for g in optimizer.param_groups for p in g["params"]]
        self._optimizers[(module_id, optimizer_name)] = (optimizer, params)

    def get_optimizer(self, module_id=None, optimizer_name="default"):
        """The named optimizer of ``module_id`` (default: this learner's own module; an
        added module's is looked up on its learner)."""
        module_id = self.module_id if module_id is None else module_id
        lr = self._module_learners().get(module_id, self)
        ent = lr._optimizers.get((module_id, optimizer_name))
        return ent[0] if ent else None

    def get_optimizers_for_module(self, module_id=None):
        module_id = self.module_id if module_id is None else module_id
        lr = self._module_learners().get(module_id, self)
        return [(n, o) for (m, n), (o, _) in lr._optimizers.items() if m == module_id]

    def get_parameters(self, module=None):
        return list((module or self.module).parameters())

    def _named_params(self):
        """name -> parameter over every registered optimizer's parameters (stable order)."""
        names = {id(p): n for n, p in self.module.named_parameters()}
        out = {}
        for (m, oname), (_, ps) in self._optimizers.items():
            for i, p in enumerate(ps):
                out.setdefault(names.get(id(p), f"{m}/{oname}/{i}"), p)
        return out

    # ---------------------------------------------------------------- multi-learner
    def _broadcast_params(self):
        import torch.distributed as dist

        if not dist.is_initialized():
            return
        with torch.no_grad():
            for t in list(self.module.parameters()) + list(self.module.buffers()):
                dist.broadcast(t.data, src=0)

    def _allreduce_grads(self, params):
        """Average the gradients of ``params`` over the learner group: one flat fp32
        all-reduce (missing gradients count as zeros, so every rank packs the same)."""
        if self.world <= 1:
            return
        import torch.distributed as dist

        if not dist.is_initialized():
            return
        flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                          .float() for p in params])
        dist.all_reduce(flat)
        flat.div_(self.world)
        o = 0
        for p in params:
            n = p.numel()
            g = flat[o:o + n].view_as(p).to(p.dtype)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
            o += n

    def _allreduce_mean(self, x: float) -> float:
        """Mean of a host scalar over the learner group (learner-side statistics that must
        stay identical on every rank)."""
        if self.world <= 1:
            return float(x)
        import torch.distributed as dist

        t = torch.tensor([float(x)], dtype=torch.float64,
                         device=self.device if self.device.type == "cuda" else "cpu")
        dist.all_reduce(t)
        return float(t) / self.world

    def _allreduce_min(self, x: int) -> int:
        if self.world <= 1:
            return int(x)
        import torch.distributed as dist

        if not dist.is_initialized():
            return int(x)
        t = torch.tensor([int(x)], dtype=torch.int64,
                         device=self.device if self.device.type == "cuda" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t)

    def _minibatch_rng(self):
        """The minibatch shuffler: created once, so a seeded learner draws a new permutation
        every epoch and iteration (the reference's MiniBatchCyclicIterator keeps its state);
        rank-offset so the learners of a group shuffle their shards independently."""
        rng = getattr(self, "_mb_rng", None)
        if rng is None:
            seed = self.config.get("seed")
            rng = self._mb_rng = np.random.default_rng(
                None if seed is None else int(seed) + 1000003 * self.rank)
        return rng

    # ---------------------------------------------------------------- the pipeline
    def update_from_batch(self, batch, *, timesteps=None, num_epochs=1, minibatch_size=None,
                          shuffle_batch_per_epoch=False, **kwargs) -> dict:
        """Gradient updates on ``batch`` (a dict of arrays / tensors with a common leading
        row axis): ``num_epochs`` passes in minibatches of ``minibatch_size`` rows (the
        whole batch by default). Returns the last update's metrics (scalars; per-row
        arrays such as ``td_error`` cover the whole batch). A module-keyed batch
        (``{module_id: batch}``) trains each of this learner's modules in it."""
        if self._is_module_batch(batch):
            return self._update_modules(batch, timesteps=timesteps, num_epochs=num_epochs,
                                        minibatch_size=minibatch_size,
                                        shuffle_batch_per_epoch=shuffle_batch_per_epoch,
                                        **kwargs)
        n = _rows(batch)
        # every update all-reduces gradients across the group, so all learners must run the
        # same number of them: agree on the smallest shard (an empty shard raises on every
        # rank together instead of leaving the others blocked in the collective)
        n_min = self._allreduce_min(n)
        if n_min == 0:
            raise ValueError(f"learner {self.rank}/{self.world}: a learner received an empty "
                             "batch shard")
        if not minibatch_size or minibatch_size >= n_min:
            res = {}
            for _ in range(max(1, num_epochs)):
                res = self._update(batch, timesteps=timesteps)
            return res
        res, per_row = {}, {}
        n_mb = n_min // minibatch_size  # minibatches per epoch, identical on every rank
        rng = self._minibatch_rng()
        for _ in range(max(1, num_epochs)):
            order = rng.permutation(n) if shuffle_batch_per_epoch else np.arange(n)
            for s in range(0, n_mb * minibatch_size, minibatch_size):
                idx = order[s:s + minibatch_size]
                res = self._update(_take_rows(batch, idx), timesteps=timesteps)
                for k, v in list(res.items()):
                    if isinstance(v, np.ndarray) and v.shape[:1] == (len(idx),):
                        per_row.setdefault(k, np.zeros((n,) + v.shape[1:], v.dtype))[idx] = v
        res.update(per_row)
        return res

    def update_from_iterator(self, iterator=None, *, timesteps=None, minibatch_size=None,
                             num_iters=None, transform=None, seed=None, **kwargs) -> dict:
        """``num_iters`` updates on batches of ``minibatch_size`` rows pulled from a
        ray_amd.data iterator (reference: learner.py update_from_iterator): this learner's
        ``streaming_split`` shard of the offline dataset. The iterator is kept across calls
        (epochs continue); ``transform`` maps each batch before the update."""
        from ray_amd.rllib.offline.offline_data import iterate_forever

        if iterator is not None and iterator is not getattr(self, "_data_it", None):
            self._data_it = iterator
            self._data_gen = iterate_forever(iterator, int(minibatch_size), seed)
        if getattr(self, "_data_gen", None) is None:
            raise ValueError("update_from_iterator needs an iterator on the first call")
        res = {}
        for _ in range(int(num_iters or 1)):
            b = next(self._data_gen)
            if transform is not None:
                b = transform(b)
            res = self.update_from_batch(b, timesteps=timesteps, **kwargs)
        return res

    def update_from_episodes(self, episodes, *, timesteps=None, **kwargs) -> dict:
        """Train on a list of SingleAgentEpisodes (the learner connector step of the
        reference: ``episodes_to_batch`` flattens them into transition rows)."""
        return self.update_from_batch(self.episodes_to_batch(episodes), timesteps=timesteps,
                                      **kwargs)

    def episodes_to_batch(self, episodes) -> dict:
        obs, nobs, act, rew, term = [], [], [], [], []
        for ep in episodes:
            o = np.asarray(ep.get_observations())
            T = len(ep.get_actions())
            obs.append(o[:T])
            nobs.append(o[1:T + 1])
            act.append(np.asarray(ep.get_actions()))
            rew.append(np.asarray(ep.get_rewards(), np.float32))
            t = np.zeros(T, np.float32)
            if ep.is_terminated and T:
                t[-1] = 1.0
            term.append(t)
        return {"obs": np.concatenate(obs), "next_obs": np.concatenate(nobs),
                "actions": np.concatenate(act), "rewards": np.concatenate(rew),
                "terminateds": np.concatenate(term)}

    def _update(self, batch, timesteps=None) -> dict:
        batch = self._convert_batch(batch)
        fwd_out = self.forward_train(batch)
        losses = self.compute_losses(fwd_out=fwd_out, batch=batch)
        grads = self.compute_gradients(losses)
        grads = self.postprocess_gradients(grads)
        self.apply_gradients(grads)
        self.updates += 1
        self.after_gradient_based_update(timesteps=timesteps)
        out = {f"{k}_loss" if not str(k).endswith("loss") else str(k): float(v.detach())
               for k, v in losses.items()}
        out["total_loss"] = float(sum(float(v.detach()) for v in losses.values()))
        out.update(self.metrics)
        return out

    def _convert_batch(self, batch) -> dict:
        out = {}
        for k, v in batch.items():
            if isinstance(v, np.ndarray):
                out[k] = torch.from_numpy(np.ascontiguousarray(v)).to(self.device)
            elif torch.is_tensor(v):
                out[k] = v.to(self.device)
            else:
                out[k] = v
        return out

    def forward_train(self, batch) -> dict:
        return self.module.forward_train(batch[Columns.OBS])

    def compute_losses(self, *, fwd_out, batch) -> dict:
        return {self.module_id: self.compute_loss_for_module(module_id=self.module_id,
                                                             config=self.config, batch=batch,
                                                             fwd_out=fwd_out)}

    def compute_loss_for_module(self, *, module_id, config, batch, fwd_out):
        raise NotImplementedError

    def compute_gradients(self, loss_per_module, **kwargs) -> dict:
        """Back-propagate and average over the learner group; returns {param name: grad}.
        Losses keyed by optimizer names go into those optimizers' parameters only."""
        named = self._named_params()
        params = list(named.values())
        for p in params:
            p.grad = None
        by_opt = {n: ps for (m, n), (_, ps) in self._optimizers.items()}
        if len(self._optimizers) > 1 and set(loss_per_module) <= set(by_opt):
            keys = list(loss_per_module)
            for i, k in enumerate(keys):
                loss_per_module[k].backward(retain_graph=i + 1 < len(keys),
                                            inputs=list(by_opt[k]))
        else:
            sum(loss_per_module.values()).backward()
        self._allreduce_grads(params)
        return {n: p.grad for n, p in named.items() if p.grad is not None}

    def postprocess_gradients(self, gradients_dict) -> dict:
        return self.postprocess_gradients_for_module(module_id=self.module_id,
                                                     config=self.config,
                                                     module_gradients_dict=gradients_dict)

    def postprocess_gradients_for_module(self, *, module_id, config, module_gradients_dict):
        """Default: ``grad_clip`` by ``grad_clip_by`` ("global_norm" (default), "norm" per
        tensor, or "value")."""
        clip = (config or {}).get("grad_clip")
        if not clip:
            return module_gradients_dict
        by = (config or {}).get("grad_clip_by", "global_norm")
        grads = [g for g in module_gradients_dict.values() if g is not None]
        if by == "value":
            for g in grads:
                g.clamp_(-clip, clip)
        elif by == "norm":
            for g in grads:
                n = g.norm()
                if n > clip:
                    g.mul_(clip / (n + 1e-6))
        else:
            torch.nn.utils.clip_grad_norm_(grads, clip)  # clips the tensors in place
        return module_gradients_dict

    def apply_gradients(self, gradients_dict):
        named = self._named_params()
        for n, g in gradients_dict.items():
            p = named.get(n)
            if p is not None and g is not p.grad:
                p.grad = g
        for opt, _ in self._optimizers.values():
            opt.step()

    def after_gradient_based_update(self, *, timesteps=None):
        """Hook after every update (target networks, schedules)."""

    # ---------------------------------------------------------------- the module set
    # Reference: rllib/core/learner/learner.py :821 add_module, :845 remove_module, :696 /
    # :714 get_module_state / set_module_state, :1308 / :1316 set_optimizer_state /
    # get_optimizer_state, :607 register_metrics. A learner owns its own module (built in
    # __init__) and any number of added ones. Each added module gets a learner of this
    # same class (same rank / world / device): its network, its optimizers (from
    # configure_optimizers_for_module) and its loss, so every algorithm's learner can grow
    # a module. A module-keyed batch ({module_id: batch}) trains every module in it, in
    # sorted module-id order, each with its own gradient all-reduce — the same order on
    # every learner of the group, so the collectives match.
    def _module_learners(self) -> dict:
        return {self.module_id: self, **(getattr(self, "_sub_learners", None) or {})}

    @property
    def module_ids(self) -> list:
        return list(self._module_learners())

    def get_module(self, module_id=None):
        lr = self._module_learners().get(module_id if module_id is not None else self.module_id)
        if lr is None:
            raise KeyError(f"no module {module_id!r} in this learner")
        return lr.module

    def add_module(self, *, module_id, module_spec=None, config_overrides=None,
                   new_should_module_be_updated=None):
        """Build and add a module. ``module_spec``: an RLModuleSpec (a user module and/or
        its spaces) or an ``(observation_space, action_space)`` tuple; missing spaces
        default to this learner's. ``config_overrides``: per-module config keys (e.g. its
        ``lr``). ``new_should_module_be_updated``: ids (or a predicate) of the modules
        that train from now on. Collective with several learners: every learner of the
        group must add it (``LearnerGroup.add_module``), which starts every copy from rank
        0's initial weights."""
        if module_id in self._module_learners():
            raise ValueError(f"module {module_id!r} already exists")
        from ray_amd.rllib.core.rl_module.rl_module import RLModuleSpec

        os_, as_ = self.observation_space, self.action_space
        cfg = dict(self.config)
        cfg.update(config_overrides or {})
        if isinstance(module_spec, (tuple, list)):
            os_, as_ = module_spec
        elif isinstance(module_spec, RLModuleSpec):
            os_ = module_spec.observation_space or os_
            as_ = module_spec.action_space or as_
            if module_spec.module_class is not None:
                cfg["_rl_module_spec"] = module_spec
        elif module_spec is not None:
            raise TypeError(f"module_spec must be an RLModuleSpec or (obs_space, act_space), "
                            f"got {type(module_spec).__name__}")
        cfg["is_multi_agent"] = bool(cfg.get("is_multi_agent"))
        sub = type(self)(cfg, os_, as_, device=self.device, rank=self.rank, world=self.world,
                         module_id=module_id)
        if not hasattr(self, "_sub_learners"):
            self._sub_learners = {}
        self._sub_learners[module_id] = sub
        if new_should_module_be_updated is not None:
            self._set_trainable_modules(new_should_module_be_updated)
        return self.module_ids

    def remove_module(self, module_id, *, new_should_module_be_updated=None):
        if module_id == self.module_id:
            raise ValueError("a learner cannot remove its own (first) module")
        sub = (getattr(self, "_sub_learners", None) or {}).pop(module_id, None)
        if sub is None:
            raise KeyError(f"no module {module_id!r} in this learner")
        sub.shutdown()
        if new_should_module_be_updated is not None:
            self._set_trainable_modules(new_should_module_be_updated)
        return self.module_ids

    def _set_trainable_modules(self, spec):
        ids = self.module_ids
        self._trainable = {m for m in ids if spec(m)} if callable(spec) else \
            set(spec) & set(ids)

    def should_module_be_updated(self, module_id) -> bool:
        tr = getattr(self, "_trainable", None)
        return tr is None or module_id in tr

    def get_module_state(self, module_ids=None) -> dict:
        """{module_id: the module's full state dict (cpu tensors: target networks and
        buffers included)}; ``module_ids`` selects."""
        lrs = self._module_learners()
        ids = lrs if module_ids is None else [m for m in lrs if m in set(module_ids)]
        return {m: {k: v.detach().cpu().clone() for k, v in lrs[m].module.state_dict().items()}
                for m in ids}

    def set_module_state(self, state: dict):
        """Load ``get_module_state`` output — or a module's EnvRunner weights
        (``get_weights`` format, e.g. an online network without its target)."""
        lrs = self._module_learners()
        for m, w in state.items():
            if m not in lrs:
                raise KeyError(f"no module {m!r} in this learner")
            lr = lrs[m]
            if set(w) == set(lr.module.state_dict()):
                lr._load_module_state_dict(w)
            else:
                lr.set_weights(w)

    def _load_module_state_dict(self, sd):
        self.module.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()})

    def _own_optimizer_state(self) -> dict:
        return {f"{m}/{n}": o.state_dict() for (m, n), (o, _) in self._optimizers.items()}

    def _load_own_optimizer_state(self, st: dict):
        for (m, n), (o, _) in self._optimizers.items():
            if f"{m}/{n}" in st:
                o.load_state_dict(st[f"{m}/{n}"])

    def get_optimizer_state(self) -> dict:
        """{module_id: {"<module>/<optimizer name>": optimizer state_dict}} over every
        module of this learner (moments, step counts: enough to resume bit-exactly)."""
        return {m: lr._own_optimizer_state() for m, lr in self._module_learners().items()}

    def set_optimizer_state(self, state: dict):
        lrs = self._module_learners()
        for m, st in state.items():
            if m not in lrs:
                raise KeyError(f"no module {m!r} in this learner")
            lrs[m]._load_own_optimizer_state(st)

    def register_metrics(self, module_id, metrics_dict: dict):
        """Metrics a loss wants reported with the update results (per module; the
        learner's own module's appear unprefixed, an added module's as ``<id>/<key>``)."""
        lr = self._module_learners().get(module_id)
        if lr is None:
            raise KeyError(f"no module {module_id!r} in this learner")
        lr.metrics.update({k: float(v.detach()) if torch.is_tensor(v) else v
                           for k, v in metrics_dict.items()})

    def register_metric(self, module_id, key: str, value) -> None:
        """One metric (reference: Learner.register_metric)."""
        self.register_metrics(module_id, {key: value})

    @property
    def distributed(self) -> bool:
        """True when this learner all-reduces with peers (a multi-learner group)."""
        return self.world > 1

    def apply(self, func, *args, **kwargs):
        """``func(self, *args, **kwargs)`` (LearnerGroup.foreach_learner's per-learner call)."""
        return func(self, *args, **kwargs)

    def compute_loss(self, *, fwd_out, batch):
        """The total loss: the sum of ``compute_losses`` over modules (old-stack name)."""
        losses = self.compute_losses(fwd_out=fwd_out, batch=batch)
        return sum(losses.values()) if isinstance(losses, dict) else losses

    def compile_results(self, *, batch, fwd_out, loss_per_module, metrics_per_module=None):
        """Per-module result dicts: the loss plus the metrics registered for the module."""
        out = {}
        for mid, loss in (loss_per_module or {}).items():
            r = {"total_loss": float(loss.detach()) if torch.is_tensor(loss) else loss}
            lr = self._module_learners().get(mid)
            if lr is not None:
                r.update(getattr(lr, "metrics", {}) or {})
            r.update((metrics_per_module or {}).get(mid, {}))
            out[mid] = r
        return out

    def filter_param_dict_for_optimizer(self, param_dict: dict, optimizer) -> dict:
        """The entries of ``param_dict`` whose tensors ``optimizer`` updates."""
        groups = getattr(optimizer, "param_groups", None)
        if groups is not None:
            ids = {id(p) for g in groups for p in g["params"]}
        else:  # a flat-buffer optimizer (FlatAdamW) updates every parameter of its buffer
            flat = getattr(optimizer, "flat", None)
            ps = flat.params() if flat is not None and callable(getattr(flat, "params", None)) \
                else self.module.parameters()
            ids = {id(p) for p in ps}
        return {k: v for k, v in param_dict.items() if id(v) in ids}

    def get_param_ref(self, param):
        """A stable reference to a parameter: its qualified name in the module."""
        for n, p in self.module.named_parameters():
            if p is param:
                return n
        return id(param)

    def additional_update(self, *, module_ids_to_update=None, timestep=None, **kwargs) -> dict:
        """Old-stack hook run after the gradient updates (reference:
        Learner.additional_update): ``additional_update_for_module`` per module."""
        mids = module_ids_to_update or self.module_ids
        return {mid: self.additional_update_for_module(module_id=mid, config=self.config,
                                                       timestep=timestep, **kwargs)
                for mid in mids}

    def additional_update_for_module(self, *, module_id, config=None, timestep=None,
                                     **kwargs) -> dict:
        return {}

    def _is_module_batch(self, batch) -> bool:
        lrs = self._module_learners()
        return isinstance(batch, dict) and bool(batch) and len(lrs) > 1 and \
            all(k in lrs and isinstance(v, dict) for k, v in batch.items())

    def _update_modules(self, batch, **kwargs) -> dict:
        lrs = self._module_learners()
        out = {}
        for m in sorted(batch, key=str):
            if not self.should_module_be_updated(m):
                continue
            # the owner's own update entry point (not this method again)
            res = lrs[m].update_from_batch(batch[m], **kwargs)
            out.update(res if m == self.module_id else {f"{m}/{k}": v for k, v in res.items()})
        return out

    # ---------------------------------------------------------------- state
    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.module.state_dict().items()}

    def set_weights(self, w):
        self.module.load_state_dict({k: torch.as_tensor(v) for k, v in w.items()})

    def get_state(self):
        return {"module": {k: v.detach().cpu() for k, v in self.module.state_dict().items()},
                "optimizers": {f"{m}/{n}": o.state_dict()
                               for (m, n), (o, _) in self._optimizers.items()},
                "updates": self.updates, "extra": self._extra_state()}

    def set_state(self, s):
        self.module.load_state_dict({k: torch.as_tensor(v) for k, v in s["module"].items()})
        for (m, n), (o, _) in self._optimizers.items():
            st = (s.get("optimizers") or {}).get(f"{m}/{n}")
            if st is not None:
                o.load_state_dict(st)
        self.updates = s.get("updates", self.updates)
        self._load_extra_state(s.get("extra") or {})

    def _extra_state(self) -> dict:
        return {}

    def _load_extra_state(self, s: dict):
        pass

    def save_state(self, path: str):
        """Checkpoint this learner (module weights, optimizer states, counters, added
        modules) into the directory ``path``: tensors and plain containers only, loaded
        back with ``torch.load(weights_only=True)`` (no code runs from the file)."""
        os.makedirs(path, exist_ok=True)
        torch.save(_plain(self.get_full_state()), os.path.join(path, "learner_state.pt"))
        return path

    def load_state(self, path: str):
        f = os.path.join(path, "learner_state.pt") if os.path.isdir(path) else path
        self.set_full_state(torch.load(f, map_location="cpu", weights_only=True))

    def get_full_state(self) -> dict:
        """This learner's state plus every added module's (``get_state`` per module)."""
        st = self.get_state()
        subs = getattr(self, "_sub_learners", None)
        if subs:
            st = dict(st, __modules__={m: lr.get_state() for m, lr in subs.items()})
        return st

    def set_full_state(self, s: dict):
        s = dict(s)
        mods = s.pop("__modules__", None) or {}
        self.set_state(s)
        for m, st in mods.items():
            sub = (getattr(self, "_sub_learners", None) or {}).get(m)
            if sub is not None:
                sub.set_state(st)

    def shutdown(self):
        pass


def _plain(x):
    """numpy values -> tensors / Python scalars, recursively, so a state file needs no
    unpickling of arbitrary classes (torch.load(weights_only=True))."""
    if isinstance(x, dict):
        return {k: _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_plain(v) for v in x)
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x))
    if isinstance(x, np.generic):
        return x.item()
    return x


def _rows(batch) -> int:
    for v in batch.values():
        if isinstance(v, (np.ndarray, torch.Tensor)) and getattr(v, "ndim", 0) >= 1:
            return int(v.shape[0])
    return 0


def _take_rows(batch, idx):
    out = {}
    n = _rows(batch)
    for k, v in batch.items():
        if isinstance(v, (np.ndarray, torch.Tensor)) and getattr(v, "ndim", 0) >= 1 and \
                v.shape[0] == n:
            out[k] = v[idx] if isinstance(v, np.ndarray) else v[torch.as_tensor(idx)]
        else:
            out[k] = v
    return out


class Learner(TorchLearner):
    """One learner (one GPU). Extension points (reference: rllib/core/learner/learner.py
    :435 configure_optimizers_for_module, :948 compute_loss_for_module):

    * ``configure_optimizers_for_module(module_id, config)`` — the default keeps the fused
      flat-buffer AdamW (HIP kernel, fp32 master + bf16 compute weights); an override
      calls ``register_optimizer(...)`` with any torch optimizer over ``self.module``'s
      parameters (then weights stay fp32).
    * ``compute_loss_for_module(module_id, config, batch, fwd_out)`` — the default is the
      fused HIP PPO loss (PPO) / the V-trace loss (IMPALA/APPO); an override gets the
      minibatch as a dict of tensors (``Columns.*`` plus ``advantages`` /
      ``value_targets``, or ``vtrace_vs`` / ``pg_advantages``) and the module's
      ``forward_train`` output, and returns the scalar loss.

    User modules, stateful modules and overridden losses run the generic (eager) SGD loop;
    the built-in module with the built-in loss keeps the captured HIP-graph step."""

    def __init__(self, config: dict, observation_space, action_space, device=None, rank=0,
                 world=1, module_id=DEFAULT_MODULE_ID):
        self.config = config
        self.observation_space, self.action_space = observation_space, action_space
        if device is None:
            device = torch.device("cuda", int(os.environ.get("RAY_AMD_LOCAL_DEVICE", "0"))) \
                if torch.cuda.is_available() and config.get("num_gpus_per_learner", 1) else \
                torch.device("cpu")
        self.device = device
        self.rank, self.world = rank, world
        self.module_id = module_id
        torch.manual_seed(config.get("seed") or 0)
        self.module = build_module(config, observation_space, action_space,
                                   module_id if config.get("is_multi_agent") else None
                                   ).to(device)
        self._builtin_module = isinstance(self.module, RLModule)
        self.stateful = bool(getattr(self.module, "is_stateful", lambda: False)()) and \
            hasattr(self.module, "forward_sequence")
        if device.type == "cuda" and self._builtin_module:
            # NHWC conv weights (FlatParams keeps the layout): no per-call weight relayout
            self.module.to(memory_format=torch.channels_last)
        self._pinned = {}
        self._optimizers = {}  # (module_id, name) -> (torch optimizer, params)
        self.configure_optimizers_for_module(module_id, config)
        from ray_amd.parallel.flat import FlatAdamW, FlatDDP, FlatParams

        # bf16 compute weights + fp32 master in the flat optimizer on GPU: no per-forward
        # autocast weight casts (they were ~30 copy kernels per SGD step). A registered
        # torch optimizer updates the parameters themselves: keep them fp32.
        bf16 = device.type == "cuda" and config.get("learner_bf16", True) and \
            not self._optimizers
        pdt = torch.bfloat16 if bf16 else torch.float32
        # grads alias .grad (same dtype as the compute weights): the whole SGD step,
        # including MIOpen's conv weight grads, stays capturable in one HIP graph
        self.flat = FlatParams(self.module, dtype=pdt, grad_dtype=pdt)
        self.ddp = FlatDDP(self.flat, bucket_mb=32.0)
        self.opt = None if self._optimizers else FlatAdamW(
            self.flat, lr=config.get("lr", 5e-5), betas=(0.9, 0.999), eps=1e-7,
            weight_decay=0.0, max_grad_norm=config.get("grad_clip"),
            grad_scale=self.ddp.grad_scale)
        self.kl_coeff = config.get("kl_coeff", 0.2)
        self.amp = device.type == "cuda" and config.get("learner_bf16", True)
        self.updates = 0
        self._custom_loss = type(self).compute_loss_for_module is not \
            Learner.compute_loss_for_module
        # an overridden gradient hook also needs the eager loop (the captured HIP-graph
        # step fuses backward, clip and AdamW)
        hooks = any(getattr(type(self), h) is not getattr(Learner, h) for h in
                    ("compute_gradients", "postprocess_gradients",
                     "postprocess_gradients_for_module", "apply_gradients"))
        self._generic = self._custom_loss or not self._builtin_module or self.stateful or \
            bool(self._optimizers) or hooks
        self.metrics = {}
        # MeanStdFilter statistics live HERE: updated over every training batch by the HIP
        # Welford kernel (obsnorm_update) and broadcast to the EnvRunners with the weights
        self.obs_filter = None
        if config.get("_learner_obs_filter"):
            from ray_amd.ops.functional import RunningMeanStd

            self.obs_filter = RunningMeanStd(observation_space.shape, device)

    # ---------------------------------------------------------------- extension API
    def configure_optimizers_for_module(self, module_id, config):
        """Default: the fused flat AdamW built in __init__ (nothing to register)."""

    def register_optimizer(self, *, module_id=DEFAULT_MODULE_ID, optimizer_name="default",
                           optimizer, params=None, lr_or_lr_schedule=None):
        params = list(params) if params is not None else \
            [p for g in optimizer.param_groups for p in g["params"]]
        self._optimizers[(module_id, optimizer_name)] = (optimizer, params)

    def get_optimizer(self, module_id=None, optimizer_name="default"):
        module_id = self.module_id if module_id is None else module_id
        lr = self._module_learners().get(module_id, self)
        ent = lr._optimizers.get((module_id, optimizer_name))
        return ent[0] if ent else lr.opt

    def get_parameters(self, module=None):
        return list((module or self.module).parameters())

    def compute_loss_for_module(self, module_id, config, batch, fwd_out):
        """Default losses: PPO (fused HIP kernel for discrete actions) or V-trace."""
        if "vtrace_vs" in batch:
            return self._vtrace_loss(batch, fwd_out)[0]
        loss, st = self._ppo_loss(fwd_out, batch[Columns.ACTION_DIST_INPUTS],
                                  batch[Columns.ACTIONS], batch[Columns.ACTION_LOGP],
                                  batch[Columns.ADVANTAGES], batch[Columns.VALUE_TARGETS])
        self._last_stats = st
        return loss

    def compute_losses(self, fwd_out, batch):
        return {self.module_id: self.compute_loss_for_module(self.module_id, self.config,
                                                             batch, fwd_out)}

    def _filter_obs(self, obs_flat, boot_obs):
        """Normalize raw observations (updating the running stats with this batch)."""
        if self.obs_filter is None:
            return obs_flat, boot_obs
        f = self.obs_filter
        if self.world > 1:  # every learner must see the same statistics: merge first
            import torch.distributed as dist

            n = torch.tensor([obs_flat.shape[0]], device=obs_flat.device, dtype=torch.float64)
            x = obs_flat.reshape(obs_flat.shape[0], -1).float()
            s1 = x.sum(0).double()
            s2 = (x.double() ** 2).sum(0)
            for t in (n, s1, s2):
                dist.all_reduce(t)
            tot = f.count + int(n.item())
            bm = (s1 / n).float()
            bv = (s2 / n - (s1 / n) ** 2).clamp_min(0).float()
            d = bm - f.mean
            f.mean = f.mean + d * (float(n) / tot)
            f.m2 = f.m2 + bv * float(n) + d * d * f.count * float(n) / tot
            f.count = tot
        else:
            f.update(obs_flat)
        return f.normalize(obs_flat), f.normalize(boot_obs)

    # ---------------------------------------------------------------- weights
    def get_weights(self):
        w = {k: v.detach().float().cpu() for k, v in self.module.state_dict().items()}
        if self.obs_filter is not None:
            w["__connector_state__"] = self.obs_filter.state_dict()
        return w

    def set_weights(self, w):
        w = dict(w)
        cs = w.pop("__connector_state__", None)
        if cs is not None and self.obs_filter is not None:
            self.obs_filter.load_state_dict(cs)
        self.module.load_state_dict({k: torch.as_tensor(v) for k, v in w.items()})
        self.flat.sync_master_from_params()

    def get_state(self):
        """Lossless learner state: the fp32 MASTER weights (not the bf16 compute copy),
        their flat layout, and the optimizer moments."""
        return {"weights": self.get_weights(),
                "master": {"p32": self.flat.p32.detach().cpu(), "names": list(self.flat.names),
                           "offsets": list(self.flat.offsets)},
                "opt": {k: v.cpu() if torch.is_tensor(v) else v
                        for k, v in self.opt.state_dict().items()} if self.opt is not None
                else None,
                "torch_opts": {f"{m}/{n}": o.state_dict()
                               for (m, n), (o, _) in self._optimizers.items()},
                "kl_coeff": self.kl_coeff,
                "obs_filter": self.obs_filter.state_dict() if self.obs_filter is not None
                else None}

    def set_state(self, s):
        if s.get("obs_filter") is not None and self.obs_filter is not None:
            self.obs_filter.load_state_dict(s["obs_filter"])
        m = s.get("master")
        if m is not None and m["names"] == list(self.flat.names) and \
                m["offsets"] == list(self.flat.offsets):
            with torch.no_grad():
                self.flat.p32.copy_(m["p32"].to(self.device))
                if self.flat.p16 is not self.flat.p32:
                    self.flat.p16.copy_(self.flat.p32)
        else:  # older checkpoint / different layout: rebuild the master from the weights
            self.set_weights(s["weights"])
        if self.opt is not None and s.get("opt") is not None:
            self.opt.load_state_dict({k: v.to(self.device) if torch.is_tensor(v) else v
                                      for k, v in s["opt"].items()})
        for (m, n), (o, _) in self._optimizers.items():
            st = (s.get("torch_opts") or {}).get(f"{m}/{n}")
            if st is not None:
                o.load_state_dict(st)
        self.kl_coeff = s.get("kl_coeff", self.kl_coeff)

    def _load_module_state_dict(self, sd):
        super()._load_module_state_dict(sd)
        self.flat.sync_master_from_params()

    def _own_optimizer_state(self) -> dict:
        st = super()._own_optimizer_state()
        if self.opt is not None:  # the fused flat AdamW (moments of the fp32 master)
            st[f"{self.module_id}/default"] = {
                k: v.detach().cpu().clone() if torch.is_tensor(v) else v
                for k, v in self.opt.state_dict().items()}
        return st

    def _load_own_optimizer_state(self, st: dict):
        super()._load_own_optimizer_state(st)
        if self.opt is not None and f"{self.module_id}/default" in st:
            self.opt.load_state_dict({k: v.to(self.device) if torch.is_tensor(v) else v
                                      for k, v in st[f"{self.module_id}/default"].items()})

    # ---------------------------------------------------------------- multi-learner agreement
    def _allreduce(self, t, op="sum"):
        """all-reduce across the learner group (no-op for a single learner)."""
        if self.world <= 1:
            return t
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.MIN if op == "min" else dist.ReduceOp.SUM)
        return t

    # ---------------------------------------------------------------- helpers
    def _fwd(self, obs):
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.amp):
            return self.module.forward_train(obs)

    def _h2d(self, x, key):
        """Host batch field -> device. Large arrays are staged through a persistent pinned
        buffer per field (multi-threaded host copy, then an async DMA), instead of
        page-locking a fresh copy of every rollout batch."""
        dev = self.device
        if not (isinstance(x, (np.ndarray, Fragments)) and dev.type == "cuda"
                and x.nbytes >= (1 << 20)):
            return _to_t(x, dev)
        if isinstance(x, np.ndarray):
            x = np.ascontiguousarray(x)
        shape, dtype = tuple(x.shape), np.dtype(x.dtype)
        ent = self._pinned.get(key)
        if ent is None or tuple(ent[0].shape) != shape or ent[0].numpy().dtype != dtype:
            ent = [torch.empty(shape, dtype=torch.from_numpy(np.empty(0, dtype)).dtype,
                               pin_memory=True), None]
            self._pinned[key] = ent
        if ent[1] is not None:
            ent[1].synchronize()  # the previous DMA out of this buffer has finished
        from ray_amd._native import _core

        dst = ent[0].numpy()
        if isinstance(x, Fragments):  # [T, B_i, ...] runner blocks -> [T, B, ...] rows
            row = int(np.prod(shape[2:], dtype=np.int64)) * dtype.itemsize
            b0 = 0
            for p in x.parts:
                bi = p.shape[1]
                _core.copy_rows(dst.reshape(-1), b0 * row, shape[1] * row, p.reshape(-1),
                                bi * row, shape[0], bi * row)
                b0 += bi
        else:
            _core.copy_into(dst, x)
        t = ent[0].to(dev, non_blocking=True)
        ent[1] = torch.cuda.Event()
        ent[1].record()
        return t

    def _values(self, obs_flat, chunk=8192):
        out = []
        with torch.no_grad():
            for i in range(0, obs_flat.shape[0], chunk):
                with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.amp):
                    out.append(self.module.value(obs_flat[i:i + chunk]).float())
        return torch.cat(out)

    def _step(self, loss):
        """One optimizer step of the generic (eager) path, through the pipeline hooks."""
        grads = self.compute_gradients({self.module_id: loss})
        grads = self.postprocess_gradients(grads)
        self.apply_gradients(grads)

    # ---- pipeline hooks on the flat-buffer layout: gradients are views of ONE buffer
    # that FlatDDP all-reduces bucket by bucket during backward; the fused AdamW kernel
    # clips by global norm on device, so the default postprocessing is a no-op there
    def compute_gradients(self, loss_per_module, **kwargs) -> dict:
        for opt, _ in self._optimizers.values():
            opt.zero_grad(set_to_none=False)
        self.flat.zero_grad()
        sum(loss_per_module.values()).backward()
        self.ddp.finish()
        return {n: (p._ra_grad if getattr(p, "_ra_grad", None) is not None else p.grad)
                for n, p in zip(self.flat.names, self.flat.params())}

    def postprocess_gradients_for_module(self, *, module_id, config, module_gradients_dict):
        if self._optimizers:  # torch optimizers: clip here (the flat AdamW clips itself)
            return super().postprocess_gradients_for_module(
                module_id=module_id, config=config, module_gradients_dict=module_gradients_dict)
        return module_gradients_dict

    def apply_gradients(self, gradients_dict):
        for n, p in zip(self.flat.names, self.flat.params()):
            g = gradients_dict.get(n)
            dst = getattr(p, "_ra_grad", None)
            if dst is None:
                dst = p.grad
            if g is not None and dst is not None and g is not dst:
                dst.copy_(g)
        if self._optimizers:
            for opt, _ in self._optimizers.values():
                opt.step()
        else:
            self.opt.step()

    def update_from_batch(self, batch, *, timesteps=None, **kwargs) -> dict:
        """PPO (GAE + epochs of minibatch SGD) or V-trace on a [T, B] rollout batch: the
        fused HIP path (loss+grad kernel, HIP-graph step) unless a pipeline hook is
        overridden, then the eager loop through the hooks. A module-keyed batch trains
        each of this learner's modules in it (``add_module``)."""
        if self._is_module_batch(batch):
            return self._update_modules(batch, timesteps=timesteps, **kwargs)
        kind = kwargs.get("kind") or self.config.get("_learner_kind", "ppo")
        return self.update_ppo(batch) if kind == "ppo" else self.update_vtrace(batch)

    # ---------------------------------------------------------------- PPO
    def update_ppo(self, batch: dict) -> dict:
        if self.stateful:
            return self._update_ppo_stateful(batch)
        c = self.config
        dev = self.device
        obs = self._h2d(batch["obs"], "obs")
        T, B = obs.shape[:2]
        rewards = _to_t(batch["rewards"], dev)
        dones = _to_t(batch["terminateds"], dev)
        acts = _to_t(batch["actions"], dev)
        old_logp = _to_t(batch["action_logp"], dev)
        old_di = _to_t(batch["action_dist_inputs"], dev)
        boot_obs = _to_t(batch["bootstrap_obs"], dev)
        obs_flat = obs.reshape((T * B,) + tuple(obs.shape[2:]))
        obs_flat, boot_obs = self._filter_obs(obs_flat, boot_obs)
        vals = self._values(obs_flat).view(T, B)
        boot_v = self._values(boot_obs)
        adv, vtarg = rf.gae(rewards, vals, dones, boot_v, c.get("gamma", 0.99),
                            c.get("lambda_", 0.95))
        adv = adv.reshape(-1)
        vtarg = vtarg.reshape(-1)
        acts = acts.reshape((T * B,) + tuple(acts.shape[2:]))
        old_logp = old_logp.reshape(-1)
        old_di = old_di.reshape(T * B, -1)
        vals = vals.reshape(-1)
        masked = "loss_mask" in batch
        if masked:
            # multi-agent padding rows (terminated, so GAE never crossed them) are dropped
            keep = _to_t(batch["loss_mask"], dev).reshape(-1).nonzero().squeeze(1)
            obs_flat, acts, old_logp, old_di, adv, vtarg, vals = (
                t.index_select(0, keep)
                for t in (obs_flat, acts, old_logp, old_di, adv, vtarg, vals))
        # advantage standardisation over the WHOLE learner group's batch; population std so
        # a 1-row shard is not NaN
        N = adv.shape[0]
        mom = self._allreduce(torch.stack([adv.sum(), (adv * adv).sum(),
                                           torch.tensor(float(N), device=dev)]).double())
        cnt = max(float(mom[2]), 1.0)
        mean = mom[0] / cnt
        std = torch.sqrt(torch.clamp(mom[1] / cnt - mean * mean, min=0.0))
        adv = ((adv - mean.float()) / (std.float() + 1e-8))
        # every rank must run the SAME number of SGD steps (each step all-reduces inside
        # backward): agree on the smallest shard and subsample to it
        if self.world > 1:
            n_common = int(self._allreduce(torch.tensor([N], device=dev), op="min")[0])
        else:
            n_common = N
        if n_common == 0:
            self.updates += 1
            return {"num_minibatches": 0, "curr_kl_coeff": self.kl_coeff}
        mb = min(int(c.get("minibatch_size", 128)), n_common)
        stats_acc = torch.zeros(6, device=dev)
        n_mb = 0
        # masked (multi-agent) batches change N every update: no graph re-capture per call
        g = None if masked or self._generic else self._ppo_graph(obs_flat, old_di, acts,
                                                                  old_logp, adv, vtarg, mb)
        if g is not None:
            # replay one captured SGD step (gather, fwd, fused loss, bwd) per minibatch;
            # the optimizer's two kernels stay eager (Adam's step count is a kernel arg)
            idx_buf, stats_buf = self._graph_io
            stats_buf.zero_()
            for _ in range(int(c.get("num_epochs", 1))):
                perm = torch.randperm(N, device=dev)[:n_common]
                for s in range(0, n_common - mb + 1, mb):
                    idx_buf.copy_(perm[s:s + mb])
                    g.replay()
                    self.ddp.finish()
                    self.opt.step()
                    n_mb += 1
            stats_acc = stats_buf
        for _ in range(int(c.get("num_epochs", 1)) if g is None else 0):
            perm = torch.randperm(N, device=dev)[:n_common]
            for s in range(0, n_common - mb + 1, mb):
                idx = perm[s:s + mb]
                out = self._fwd(obs_flat[idx])
                if self._generic:
                    mbatch = {Columns.OBS: obs_flat[idx], Columns.ACTIONS: acts[idx],
                              Columns.ACTION_LOGP: old_logp[idx],
                              Columns.ACTION_DIST_INPUTS: old_di[idx],
                              Columns.ADVANTAGES: adv[idx], Columns.VALUE_TARGETS: vtarg[idx],
                              Columns.VF_PREDS: vals[idx]}
                    self._last_stats = None
                    loss = self.compute_loss_for_module(self.module_id, c, mbatch, out)
                    st = self._last_stats if self._last_stats is not None else \
                        torch.stack([loss.detach().float()] + [torch.zeros((), device=dev)] * 5)
                else:
                    loss, st = self._ppo_loss(out, old_di[idx], acts[idx], old_logp[idx],
                                              adv[idx], vtarg[idx])
                self._step(loss)
                stats_acc += st.detach()
                n_mb += 1
        stats = (stats_acc / max(1, n_mb)).tolist()
        kl = stats[4]
        if c.get("use_kl_loss", True) and c.get("kl_target"):
            if kl > 2.0 * c["kl_target"]:
                self.kl_coeff *= 1.5
            elif kl < 0.5 * c["kl_target"]:
                self.kl_coeff *= 0.5
        self.updates += 1
        return {"total_loss": stats[0], "policy_loss": stats[1], "vf_loss": stats[2],
                "entropy": stats[3], "mean_kl_loss": kl, "clip_frac": stats[5],
                "curr_kl_coeff": self.kl_coeff, "num_minibatches": n_mb,
                "vf_explained_var": _explained_var(vtarg, vals)}

    def _update_ppo_stateful(self, batch: dict) -> dict:
        """PPO for a stateful (recurrent) module over time-major [T, B] fragments: values
        and the loss are computed by unrolling the module through each fragment from its
        recorded ``state_in`` (state zeroed where an episode starts: ``resets``);
        minibatches are whole sequences (columns), ``minibatch_size // T`` at a time."""
        c = self.config
        dev = self.device
        m = self.module
        obs = _to_t(batch["obs"], dev)
        T, B = obs.shape[:2]
        rewards = _to_t(batch["rewards"], dev)
        dones = _to_t(batch["terminateds"], dev)
        acts = _to_t(batch["actions"], dev)
        old_logp = _to_t(batch["action_logp"], dev)
        old_di = _to_t(batch["action_dist_inputs"], dev)
        boot_obs = _to_t(batch["bootstrap_obs"], dev)
        h0 = _to_t(batch["state_in_h"], dev).float()
        c0 = _to_t(batch["state_in_c"], dev).float()
        resets = _to_t(batch["resets"], dev).float()
        with torch.no_grad():
            _, vals, (hT, cT) = m.forward_sequence(obs, h0, c0, resets)
            keep = (1.0 - dones[-1].float())[:, None]
            _, boot_v, _ = m.step(boot_obs, {"h": hT * keep, "c": cT * keep})
        adv, vtarg = rf.gae(rewards.float(), vals.float(), dones.float(), boot_v.float(),
                            c.get("gamma", 0.99), c.get("lambda_", 0.95))
        N = adv.numel()
        mom = self._allreduce(torch.stack([adv.sum(), (adv * adv).sum(),
                                           torch.tensor(float(N), device=dev)]).double())
        cnt = max(float(mom[2]), 1.0)
        mean = mom[0] / cnt
        std = torch.sqrt(torch.clamp(mom[1] / cnt - mean * mean, min=0.0))
        adv = (adv - mean.float()) / (std.float() + 1e-8)
        n_common = int(self._allreduce(torch.tensor([B], device=dev), op="min")[0]) \
            if self.world > 1 else B
        seq_mb = max(1, min(n_common, int(c.get("minibatch_size", 128)) // T))
        stats_acc = torch.zeros(6, device=dev)
        n_mb = 0
        for _ in range(int(c.get("num_epochs", 1))):
            perm = torch.randperm(B, device=dev)[:n_common]
            for s in range(0, n_common - seq_mb + 1, seq_mb):
                cols = perm[s:s + seq_mb]
                logits, v, _ = m.forward_sequence(obs[:, cols], h0[cols], c0[cols],
                                                  resets[:, cols])
                n = T * cols.numel()
                out = {Columns.ACTION_DIST_INPUTS: logits.reshape(n, -1),
                       Columns.VF_PREDS: v.reshape(n)}
                mbatch = {Columns.OBS: obs[:, cols].reshape((n,) + tuple(obs.shape[2:])),
                          Columns.ACTIONS: acts[:, cols].reshape((n,) + tuple(acts.shape[2:])),
                          Columns.ACTION_LOGP: old_logp[:, cols].reshape(n),
                          Columns.ACTION_DIST_INPUTS: old_di[:, cols].reshape(n, -1),
                          Columns.ADVANTAGES: adv[:, cols].reshape(n),
                          Columns.VALUE_TARGETS: vtarg[:, cols].reshape(n),
                          Columns.VF_PREDS: vals[:, cols].reshape(n)}
                self._last_stats = None
                loss = self.compute_loss_for_module(self.module_id, c, mbatch, out)
                st = self._last_stats if self._last_stats is not None else \
                    torch.stack([loss.detach().float()] + [torch.zeros((), device=dev)] * 5)
                self._step(loss)
                stats_acc += st.detach()
                n_mb += 1
        stats = (stats_acc / max(1, n_mb)).tolist()
        kl = stats[4]
        if c.get("use_kl_loss", True) and c.get("kl_target"):
            if kl > 2.0 * c["kl_target"]:
                self.kl_coeff *= 1.5
            elif kl < 0.5 * c["kl_target"]:
                self.kl_coeff *= 0.5
        self.updates += 1
        return {"total_loss": stats[0], "policy_loss": stats[1], "vf_loss": stats[2],
                "entropy": stats[3], "mean_kl_loss": kl, "curr_kl_coeff": self.kl_coeff,
                "num_minibatches": n_mb, "vf_explained_var": _explained_var(
                    vtarg.reshape(-1), vals.reshape(-1))}

    def _ppo_graph(self, obs, old_di, acts, old_logp, adv, vtarg, mb):
        """HIP graph of one PPO SGD step over static full-batch buffers (the minibatch
        is gathered inside the graph from a static index buffer). Re-captured when the
        batch shape or the adaptive KL coefficient (a kernel scalar) changes. Single
        learner only: multi-learner steps all-reduce inside backward."""
        if (self.device.type != "cuda" or self.world > 1
                or not self.config.get("learner_cuda_graph", True)
                or getattr(self, "_graph_failed", False)):
            return None
        packed = (self.module.discrete and obs.dtype == torch.uint8 and obs.dim() >= 2
                  and obs[0].numel() % 16 == 0 and old_di.shape[-1] <= 64)
        if packed:
            src = (obs, rf.ppo_pack(old_di, acts, old_logp, adv, vtarg))
        else:
            src = (obs, old_di, acts, old_logp, adv, vtarg)
        # the packed graph reads the KL coefficient from device memory: no re-capture when
        # the adaptive coefficient moves
        key = (mb, None if packed else self.kl_coeff, packed) + tuple(
            (tuple(t.shape), t.dtype) for t in src)
        if packed:
            if getattr(self, "_kl_dev", None) is None:
                self._kl_dev = torch.zeros(1, device=self.device)
            c = self.config
            self._kl_dev.fill_(self.kl_coeff if c.get("use_kl_loss", True) else 0.0)
        if getattr(self, "_graph_key", None) == key:
            for d, s in zip(self._graph_bufs, src):
                d.copy_(s)
            return self._graph
        self._graph = None
        try:
            self._graph_packed = packed
            self._graph = self._capture_ppo_graph(src, mb, packed)
            self._n_captures = getattr(self, "_n_captures", 0) + 1
            self._graph_key = key
        except Exception as e:  # noqa: BLE001
            import warnings

            warnings.warn(f"PPO learner graph capture failed ({e!r}); running eagerly")
            self._graph_failed = True
            torch.cuda.synchronize()
            self.flat.zero_grad()
        return self._graph

    def _capture_ppo_graph(self, src, mb, packed=False):
        dev = self.device
        self._graph_bufs = bufs = [torch.empty_like(t) for t in src]
        for d, s in zip(bufs, src):
            d.copy_(s)
        idx = torch.zeros(mb, dtype=torch.long, device=dev)
        stats = torch.zeros(6, device=dev)
        self._graph_io = (idx, stats)
        params = self.flat.params()
        grads = [p._ra_grad for p in params]
        # the upstream gradient of the loss handle: the graph reads it by address, so it
        # must outlive this call (a freed scalar is reused by later allocations)
        self._graph_one = one = torch.ones((), device=dev)
        c = self.config
        kl_c = self.kl_coeff if c.get("use_kl_loss", True) else 0.0

        if packed:
            obs, aux = bufs
            m = self.module
            # the fused heads kernel needs a shared encoder and bf16 heads on the GPU
            fused_heads = (m.vf_encoder is None and self.amp
                           and m.pi.weight.dtype == torch.bfloat16
                           and m.encoder.out_dim % 8 == 0 and m.encoder.out_dim <= 1024
                           and m.pi.weight.shape[0] <= 18)

            def body():
                # minibatch frames read by the first conv kernel straight from the uint8
                # batch (gather + /255 fused into its loads); behaviour fields
                # read by the loss kernel straight from the packed table through `idx`
                # (stats accumulate in-kernel); gradients come back from autograd.grad and
                # land in the flat buffer in one multi-tensor copy instead of one
                # AccumulateGrad add per parameter (the fused bias kernels write their
                # bias gradients into the zeroed buffer directly)
                self.flat.g.zero_()
                hp = dict(clip=c.get("clip_param", 0.3), vf_clip=c.get("vf_clip_param", 10.0),
                          vf_coeff=c.get("vf_loss_coeff", 1.0),
                          ent_coeff=c.get("entropy_coeff", 0.0), kl_coeff=kl_c, has_old=True,
                          kl_dev=self._kl_dev)
                m = self.module
                with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=self.amp):
                    if fused_heads:  # heads + loss in one kernel over the encoder output
                        h = m._encode(m.encoder, m._flat(obs), idx)
                    else:
                        out = m.forward_train(obs, idx=idx)
                if fused_heads:
                    loss = rf.ppo_heads_loss(h, m.pi.weight, m.pi.bias, m.vf.weight, m.vf.bias,
                                             aux, idx, stats, **hp)
                else:
                    loss = rf.ppo_loss_packed(out["action_dist_inputs"], out["vf_preds"], aux,
                                              idx, stats, **hp)
                gs = torch.autograd.grad(loss, params, grad_outputs=one, allow_unused=True)
                dst = [g for g, x in zip(grads, gs) if x is not None]
                src_ = [x for x in gs if x is not None]
                if dst:
                    torch._foreach_copy_(dst, src_)
        else:
            obs, old_di, acts, old_logp, adv, vtarg = bufs

            def body():
                self.flat.zero_grad()
                out = self._fwd(obs.index_select(0, idx))
                loss, st = self._ppo_loss(out, old_di.index_select(0, idx),
                                          acts.index_select(0, idx),
                                          old_logp.index_select(0, idx), adv.index_select(0, idx),
                                          vtarg.index_select(0, idx))
                loss.backward()
                stats.add_(st.detach())

        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(3):  # warm kernels and solver choices; no optimizer step
                body()
        torch.cuda.current_stream(dev).wait_stream(side)
        try:  # the warm stream's GEMM workspace is not baked into the graph
            from ray_amd.ops import lt

            lt.release_stream(side)
        except (OSError, RuntimeError, AttributeError):
            pass
        from ray_amd.ops.graph_lock import CAPTURE_LOCK

        graph = torch.cuda.CUDAGraph()
        with CAPTURE_LOCK, torch.cuda.graph(graph):  # an in-process policy server waits
            body()
        self.flat.zero_grad()
        return graph

    def _ppo_loss(self, out, old_di, acts, old_logp, adv, vtarg):
        c = self.config
        kl_c = self.kl_coeff if c.get("use_kl_loss", True) else 0.0
        logits = out["action_dist_inputs"]
        v = out["vf_preds"]
        if self.module.discrete:  # the fused kernel reads bf16 heads directly
            return rf.ppo_loss(logits, old_di, acts, old_logp, adv, v, vtarg,
                               clip=c.get("clip_param", 0.3), vf_clip=c.get("vf_clip_param", 10.0),
                               vf_coeff=c.get("vf_loss_coeff", 1.0),
                               ent_coeff=c.get("entropy_coeff", 0.0), kl_coeff=kl_c)
        # DiagGaussian (continuous) path
        logits, v = logits.float(), v.float()
        mean, log_std = logits.chunk(2, -1)
        logp = gaussian_logp(acts, mean, log_std)
        ratio = torch.exp(logp - old_logp)
        clip = c.get("clip_param", 0.3)
        surr = torch.minimum(adv * ratio, adv * ratio.clamp(1 - clip, 1 + clip))
        om, ols = old_di.float().chunk(2, -1)
        ols = ols.clamp(-20, 2)
        ls = log_std.clamp(-20, 2)
        kl = (ls - ols + (ols.exp() ** 2 + (om - mean) ** 2) / (2 * ls.exp() ** 2) - 0.5).sum(-1)
        ent = gaussian_entropy(log_std)
        vf = ((v - vtarg) ** 2).clamp(0, c.get("vf_clip_param", 10.0))
        total = (-surr + c.get("vf_loss_coeff", 1.0) * vf - c.get("entropy_coeff", 0.0) * ent
                 + kl_c * kl).mean()
        cf = ((ratio < 1 - clip) | (ratio > 1 + clip)).float().mean()
        st = torch.stack([total.detach(), -surr.mean().detach(), vf.mean().detach(),
                          ent.mean().detach(), kl.mean().detach(), cf])
        return total, st

    # ---------------------------------------------------------------- IMPALA / APPO
    def update_vtrace(self, batch: dict) -> dict:
        c = self.config
        dev = self.device
        obs = self._h2d(batch["obs"], "obs")
        T, B = obs.shape[:2]
        rewards = _to_t(batch["rewards"], dev)
        dones = _to_t(batch["terminateds"], dev)
        acts = _to_t(batch["actions"], dev)
        beh_logp = _to_t(batch["action_logp"], dev)
        boot_obs = _to_t(batch["bootstrap_obs"], dev)
        obs_flat = obs.reshape((T * B,) + tuple(obs.shape[2:]))
        obs_flat, boot_obs = self._filter_obs(obs_flat, boot_obs)
        out = self._fwd(obs_flat)
        logits = out["action_dist_inputs"].float()
        v = out["vf_preds"].float().view(T, B)
        with torch.no_grad():
            boot_v = self._values(boot_obs)
        lp_all = torch.log_softmax(logits, -1)
        tgt_logp = lp_all.gather(-1, acts.reshape(-1, 1)).view(T, B)
        disc = c.get("gamma", 0.99) * (1.0 - dones)
        with torch.no_grad():
            vs, pg_adv = rf.vtrace(tgt_logp.detach() - beh_logp, disc, rewards, v.detach(), boot_v,
                                   c.get("vtrace_clip_rho_threshold", 1.0), 1.0,
                                   c.get("vtrace_clip_pg_rho_threshold", 1.0))
        vb = {Columns.OBS: obs_flat, Columns.ACTIONS: acts.reshape(-1) if acts.dim() == 2
              else acts.reshape((T * B,) + tuple(acts.shape[2:])),
              Columns.ACTION_LOGP: beh_logp.reshape(-1), "vtrace_vs": vs.reshape(-1),
              "pg_advantages": pg_adv.reshape(-1), "_T": T, "_B": B}
        if "loss_mask" in batch:  # multi-agent padding rows: excluded from every term
            vb[Columns.LOSS_MASK] = _to_t(batch["loss_mask"], dev).float().reshape(-1)
        out = dict(out)
        if self._custom_loss:
            self._vt_stats = None
            loss = self.compute_loss_for_module(self.module_id, c, vb, out)
            pg = vf = ent = loss.detach()
        else:
            loss, (pg, vf, ent) = self._vtrace_loss(vb, out)
        self._step(loss)
        self.updates += 1
        return {"total_loss": float(loss.detach()), "pi_loss": float(pg),
                "vf_loss": float(vf), "entropy": float(ent)}

    def _vtrace_loss(self, vb, out):
        """IMPALA / APPO loss over flat [T*B] rows given V-trace targets (vtrace_vs) and
        policy-gradient advantages (pg_advantages)."""
        c = self.config
        logits = out[Columns.ACTION_DIST_INPUTS].float()
        v = out[Columns.VF_PREDS].float().reshape(-1)
        lp_all = torch.log_softmax(logits, -1)
        tgt_logp = lp_all.gather(-1, vb[Columns.ACTIONS].reshape(-1, 1).long())[:, 0]
        beh_logp = vb[Columns.ACTION_LOGP]
        pg_adv, vs = vb["pg_advantages"], vb["vtrace_vs"]
        m = vb.get(Columns.LOSS_MASK)
        if m is not None:
            inv = 1.0 / m.sum().clamp_min(1.0)

            def mean(x):
                return (x * m).sum() * inv
        else:
            def mean(x):
                return x.mean()
        if c.get("appo", False):
            ratio = torch.exp(tgt_logp - beh_logp)
            clip = c.get("clip_param", 0.4)
            pg = -mean(torch.minimum(pg_adv * ratio, pg_adv * ratio.clamp(1 - clip, 1 + clip)))
        else:
            pg = -mean(tgt_logp * pg_adv)
        vf = 0.5 * mean((vs - v) ** 2)
        ent = mean(-(lp_all.exp() * lp_all).sum(-1))
        loss = pg + c.get("vf_loss_coeff", 0.5) * vf - c.get("entropy_coeff", 0.01) * ent
        return loss, (pg.detach(), vf.detach(), ent.detach())


def _learner_cls(config):
    """``config.training(learner_class=...)``: a Learner subclass (custom losses /
    optimizers); default Learner."""
    return config.get("learner_class") or Learner


# reference class names (algorithms/{ppo,impala,appo}/torch/*_torch_learner.py): one
# MI355X learner serves all three; TorchLearner is the generic pipeline base above
PPOTorchLearner = Learner
IMPALATorchLearner = Learner
APPOTorchLearner = Learner


def _explained_var(y, pred):
    vy = torch.var(y)
    return float(1 - torch.var(y - pred) / (vy + 1e-8))


class LearnerActor:
    """One learner process per GPU; a LearnerGroup of these all-reduces gradients on RCCL."""

    def __init__(self, config, observation_space, action_space, rank, world):
        self.config = config
        self.args = (observation_space, action_space, rank, world)
        self.learner = None

    def setup(self):
        obs_space, act_space, rank, world = self.args
        self.learner = _learner_cls(self.config)(self.config, obs_space, act_space, rank=rank,
                                                 world=world)
        return True

    def update(self, kind, batches):
        b = concat_batches(batches) if isinstance(batches, list) else batches
        return self.learner.update_ppo(b) if kind == "ppo" else self.learner.update_vtrace(b)

    def get_weights(self):
        return self.learner.get_weights()

    def set_weights(self, w):
        self.learner.set_weights(w)

    def get_state(self):
        return self.learner.get_state()

    def set_state(self, s):
        self.learner.set_state(s)


class LearnerGroup:
    """The learners of one module (reference: rllib/core/learner/learner_group.py):
    ``num_learners=0`` -> one local learner in the algorithm process; ``N > 0`` -> N learner
    actors (one GPU each) joined in one torch process group (RCCL on GPUs, gloo on CPUs),
    each training on its 1/N share of every batch with gradients averaged in
    ``compute_gradients``. ``learner_class`` (or ``config["learner_class"]``) picks the
    algorithm's Learner (PPO/IMPALA: the fused HIP ``Learner``; DQN, SAC, CQL, MARWIL/BC:
    their ``TorchLearner`` subclasses)."""

    def __init__(self, config: dict, observation_space, action_space,
                 module_id=DEFAULT_MODULE_ID, learner_class=None):
        self.config = config
        self.learner_class = config.get("learner_class") or learner_class or Learner
        n = int(config.get("num_learners", 0))
        self.remote = n > 0
        if not self.remote:
            self.local = self.learner_class(config, observation_space, action_space,
                                            module_id=module_id)
            self.actors = []
            return
        import ray_amd as ray
        from ray_amd.train._internal.worker_group import WorkerGroup
        from ray_amd.train.torch.config import TorchConfig, _TorchBackend

        ngpu = config.get("num_gpus_per_learner", 1)
        res = {"CPU": 1}
        if ngpu:
            res["GPU"] = ngpu

        class _LW(LearnerActor):
            pass

        self.wg = WorkerGroup(n, res)
        # learner_backend: process-group backend override (default: RCCL on GPU learners,
        # gloo on CPU); "gloo" lets several GPU learners share one device in tests
        _TorchBackend().on_start(self.wg, TorchConfig(backend=config.get("learner_backend")))
        self.actors = self.wg.workers
        ray.get([a.execute.remote(_make_learner, config, observation_space, action_space, i, n,
                                  module_id, self.learner_class)
                 for i, a in enumerate(self.actors)])
        self.local = None

    @property
    def is_local(self) -> bool:
        return not self.remote

    @property
    def is_remote(self) -> bool:
        return bool(self.remote)

    def async_update(self, batch, **kwargs):
        """Old-stack name of ``update_from_batch(async_update=True)``."""
        return self.update_from_batch(batch, async_update=True, **kwargs)

    def additional_update(self, **kwargs):
        """Run every learner's ``additional_update``; the first learner's results."""
        return self._all("additional_update", **kwargs)[0]

    def get_stats(self) -> dict:
        return {"num_learners": len(self.actors) if self.remote else 1,
                "is_local": self.is_local, "module_ids": sorted(self.get_module_state().keys())}

    def load_module_state(self, *, rl_module_ckpt_dirs=None, modules_to_load=None,
                          marl_module_ckpt_dir=None):
        """Module weights from weights-only files: ``rl_module_ckpt_dirs`` maps module ids
        to a directory holding ``module_state.pt`` (or the file itself);
        ``marl_module_ckpt_dir`` holds ``<module_id>/module_state.pt`` for every module
        (filtered by ``modules_to_load``)."""
        import os as _os

        def load(path):
            f = path if _os.path.isfile(path) else _os.path.join(path, "module_state.pt")
            return torch.load(f, weights_only=True, map_location="cpu")

        state = {}
        if marl_module_ckpt_dir:
            for mid in sorted(_os.listdir(marl_module_ckpt_dir)):
                if modules_to_load is None or mid in modules_to_load:
                    state[mid] = load(_os.path.join(marl_module_ckpt_dir, mid))
        for mid, path in (rl_module_ckpt_dirs or {}).items():
            state[mid] = load(path)
        if state:
            self.set_module_state(state)

    def update_from_batch(self, batch, *, async_update=False, timesteps=None, **kwargs):
        """One update step on ``batch`` (rows split evenly over the learners; per-row
        outputs such as ``td_error`` come back in row order, scalars averaged).
        ``async_update=True`` returns pending results (``collect_async``) instead."""
        if not self.remote:
            return self.local.update_from_batch(batch, timesteps=timesteps, **kwargs)
        import ray_amd as ray

        n = len(self.actors)
        if batch and all(isinstance(v, dict) for v in batch.values()):  # module-keyed
            per = {m: _split_rows(b, n) for m, b in batch.items()}
            shards = [{m: per[m][i] for m in batch} for i in range(n)]
            rows = [min(_rows(b) for b in sh.values()) for sh in shards]
        else:
            shards = _split_rows(batch, n)
            rows = [_rows(sh) for sh in shards]
        if min(rows) == 0:
            raise ValueError(f"a batch of {_rows(batch) if shards else 0} rows cannot feed "
                             f"{n} learners: every learner needs at least one row")
        refs = [a.execute.remote(_learner_call_kw, "update_from_batch", (sh,),
                                 dict(kwargs, timesteps=timesteps))
                for a, sh in zip(self.actors, shards)]
        if async_update:
            return refs
        return _reduce_results(ray.get(refs))

    def update_from_episodes(self, episodes, *, async_update=False, timesteps=None, **kwargs):
        """One update step on a list of episodes, split across the learners by rows: the
        longest episodes first, each to the learner with the fewest rows so far (the
        learners then agree on a common minibatch count, see ``update_from_batch``)."""
        if not self.remote:
            return self.local.update_from_episodes(episodes, timesteps=timesteps, **kwargs)
        import ray_amd as ray

        n = len(self.actors)
        if len(episodes) < n:
            raise ValueError(f"{len(episodes)} episodes cannot feed {n} learners: every "
                             "learner needs at least one")
        shards, rows = [[] for _ in range(n)], [0] * n
        for ep in sorted(episodes, key=len, reverse=True):
            i = rows.index(min(rows))
            shards[i].append(ep)
            rows[i] += len(ep)
        refs = [a.execute.remote(_learner_call_kw, "update_from_episodes", (shards[i],),
                                 dict(kwargs, timesteps=timesteps))
                for i, a in enumerate(self.actors)]
        if async_update:
            return refs
        return _reduce_results(ray.get(refs))

    def update_from_iterator(self, iterators=None, *, num_iters=1, minibatch_size=None,
                             transform=None, seed=None, timesteps=None, **kwargs):
        """Each learner actor trains ``num_iters`` updates on batches of ``minibatch_size``
        rows pulled from its own data shard (``iterators``: one per learner, e.g.
        ``Dataset.streaming_split(n, equal=True)``; passed once, kept by the learners).
        Equal shards + a fixed update count keep the learners' gradient all-reduces in
        step. Returns the rank-averaged metrics."""
        if not self.remote:
            it = iterators[0] if isinstance(iterators, (list, tuple)) else iterators
            return self.local.update_from_iterator(
                it, num_iters=num_iters, minibatch_size=minibatch_size, transform=transform,
                seed=seed, timesteps=timesteps, **kwargs)
        import ray_amd as ray

        its = list(iterators) if iterators is not None else [None] * len(self.actors)
        if len(its) != len(self.actors):
            raise ValueError(f"{len(its)} iterators for {len(self.actors)} learners")
        refs = [a.execute.remote(_learner_call_kw, "update_from_iterator", (it,), dict(
                    kwargs, num_iters=num_iters, minibatch_size=minibatch_size,
                    transform=transform, seed=None if seed is None else seed + i,
                    timesteps=timesteps))
                for i, (a, it) in enumerate(zip(self.actors, its))]
        return _reduce_results(_get_fail_fast(refs))

    def foreach_learner(self, func, **kwargs) -> list:
        """``func(learner, **kwargs)`` on every learner (local or remote), results in rank
        order (reference: learner_group.py:613)."""
        if not self.remote:
            return [func(self.local, **kwargs)]
        import ray_amd as ray

        return ray.get([a.execute.remote(_learner_apply, func, kwargs) for a in self.actors])

    def save_state(self, path: str):
        """Rank 0's learner state into directory ``path`` (all ranks hold the same)."""
        if not self.remote:
            return self.local.save_state(path)
        import ray_amd as ray

        st = ray.get(self.actors[0].execute.remote(_learner_call, "get_full_state"))
        os.makedirs(path, exist_ok=True)
        torch.save(_plain(st), os.path.join(path, "learner_state.pt"))
        return path

    def load_state(self, path: str):
        f = os.path.join(path, "learner_state.pt") if os.path.isdir(path) else path
        st = torch.load(f, map_location="cpu", weights_only=True)
        if not self.remote:
            return self.local.set_full_state(st)
        import ray_amd as ray

        ray.get([a.execute.remote(_learner_call, "set_full_state", st) for a in self.actors])

    # ---------------------------------------------------------------- the module set
    # reference: rllib/core/learner/learner_group.py:494 add_module, :520 remove_module,
    # get/set_module_state, get/set_optimizer_state. Every learner of the group runs the
    # call (adding a module is collective: its initial weights come from rank 0).
    def _all(self, name, *args, **kwargs):
        if not self.remote:
            return [getattr(self.local, name)(*args, **kwargs)]
        import ray_amd as ray

        return ray.get([a.execute.remote(_learner_call_kw, name, args, kwargs)
                        for a in self.actors])

    def add_module(self, *, module_id, module_spec=None, config_overrides=None,
                   new_should_module_be_updated=None):
        return self._all("add_module", module_id=module_id, module_spec=module_spec,
                         config_overrides=config_overrides,
                         new_should_module_be_updated=new_should_module_be_updated)[0]

    def remove_module(self, module_id, *, new_should_module_be_updated=None):
        return self._all("remove_module", module_id,
                         new_should_module_be_updated=new_should_module_be_updated)[0]

    def get_module_state(self, module_ids=None) -> dict:
        return self._all("get_module_state", module_ids)[0] if not self.remote else \
            self._rank0("get_module_state", module_ids)

    def set_module_state(self, state: dict):
        self._all("set_module_state", state)

    def get_optimizer_state(self) -> dict:
        return self._all("get_optimizer_state")[0] if not self.remote else \
            self._rank0("get_optimizer_state")

    def set_optimizer_state(self, state: dict):
        self._all("set_optimizer_state", state)

    def _rank0(self, name, *args):
        import ray_amd as ray

        return ray.get(self.actors[0].execute.remote(_learner_call_kw, name, args, {}))

    def sync_target(self):
        """Off-policy learners: copy the online networks into their targets."""
        self.foreach_learner(lambda lr: getattr(lr, "sync_target", lambda: None)())

    def update(self, kind, batches):
        if not self.remote:
            lazy = ("obs",) if self.local.device.type == "cuda" else ()
            b = concat_batches(batches, lazy) if isinstance(batches, list) else batches
            return self.local.update_ppo(b) if kind == "ppo" else self.local.update_vtrace(b)
        import ray_amd as ray

        n = len(self.actors)
        # split the env (column) axis of the whole batch evenly: shards differ by at most
        # one column whatever the runner / learner counts (the learners additionally agree
        # on a common minibatch count, see Learner.update_ppo)
        whole = concat_batches(batches) if isinstance(batches, list) else batches
        shards = [_split_b(whole, n, i) for i in range(n)]
        res = ray.get([a.execute.remote(_learner_update, kind, s)
                       for a, s in zip(self.actors, shards)])
        return res[0]

    def update_from_refs(self, kind, refs, async_update=False):
        """Remote learners pull their share of the sample batches straight from the object
        store (ObjectRefs assigned round-robin, at least one per learner): the driver never
        fetches frames (reference: impala.py:130,194 — batches go to the learners, not
        through the algorithm). async_update: return the per-learner result refs instead
        of waiting (collect with ``collect_async``)."""
        import ray_amd as ray

        n = len(self.actors)
        if not self.remote or len(refs) < n:
            batches = ray.get(list(refs))
            return self.update(kind, batches)
        shares = [refs[i::n] for i in range(n)]
        out = [a.execute.remote(_learner_update_refs, kind, sh)
               for a, sh in zip(self.actors, shares)]
        if async_update:
            return out
        return ray.get(out)[0]

    @staticmethod
    def collect_async(pending, block=False):
        """Stats of an async update when it finished (None while running)."""
        import ray_amd as ray

        if not pending:
            return None
        ready, _ = ray.wait(list(pending), num_returns=len(pending),
                            timeout=None if block else 0)
        if len(ready) < len(pending):
            return None
        return ray.get(list(pending))[0]

    def get_weights(self):
        if not self.remote:
            return self.local.get_weights()
        import ray_amd as ray

        return ray.get(self.actors[0].execute.remote(_learner_call, "get_weights"))

    def set_weights(self, w):
        if not self.remote:
            return self.local.set_weights(w)
        import ray_amd as ray

        ray.get([a.execute.remote(_learner_call, "set_weights", w) for a in self.actors])

    def get_state(self):
        """Rank 0's learner state, added modules included (all ranks hold the same)."""
        if not self.remote:
            return self.local.get_full_state()
        import ray_amd as ray

        return ray.get(self.actors[0].execute.remote(_learner_call, "get_full_state"))

    def set_state(self, s):
        if not self.remote:
            return self.local.set_full_state(s)
        import ray_amd as ray

        ray.get([a.execute.remote(_learner_call, "set_full_state", s) for a in self.actors])

    def update_modules(self, kind, per_module: dict) -> dict:
        """One PPO / V-trace update of several modules of this group's learners:
        ``per_module`` = {module_id: list of rollout batches}; returns {module_id: stats}
        (rank 0's). Modules train in sorted id order on every learner."""
        if not self.remote:
            lrs = self.local._module_learners()
            lazy = ("obs",) if self.local.device.type == "cuda" else ()
            out = {}
            for m in sorted(per_module, key=str):
                bs = per_module[m]
                b = concat_batches(bs, lazy) if isinstance(bs, list) else bs
                out[m] = lrs[m].update_ppo(b) if kind == "ppo" else lrs[m].update_vtrace(b)
            return out
        import ray_amd as ray

        n = len(self.actors)
        whole = {m: concat_batches(bs) if isinstance(bs, list) else bs
                 for m, bs in per_module.items()}
        shards = [{m: _split_b(b, n, i) for m, b in whole.items()} for i in range(n)]
        res = ray.get([a.execute.remote(_learner_update_modules, kind, sh)
                       for a, sh in zip(self.actors, shards)])
        return res[0]

    def shutdown(self):
        if self.remote:
            self.wg.shutdown()


_LEARNER = None


def _make_learner(config, obs_space, act_space, rank, world, module_id=DEFAULT_MODULE_ID,
                  learner_class=None):
    global _LEARNER
    cls = learner_class or _learner_cls(config)
    _LEARNER = cls(config, obs_space, act_space, rank=rank, world=world, module_id=module_id)
    return True


def _get_fail_fast(refs):
    """ray.get of every learner's result, raising the first learner error at once: the
    other learners may be blocked in a collective that the failed one never joins."""
    import ray_amd as ray

    pending = list(refs)
    while pending:
        ready, pending = ray.wait(pending, num_returns=1)
        ray.get(ready)  # raises the learner's error
    return ray.get(list(refs))


def _learner_call_kw(name, args, kwargs):
    return getattr(_LEARNER, name)(*args, **kwargs)


def _learner_apply(func, kwargs):
    return func(_LEARNER, **kwargs)


def _split_rows(batch, n):
    """Row shards of a dict batch (arrays with the common leading row axis are split,
    everything else is replicated)."""
    rows = _rows(batch)
    idx = np.array_split(np.arange(rows), n)
    out = []
    for ix in idx:
        sh = {}
        for k, v in batch.items():
            if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] == rows:
                sh[k] = v[ix[0]:ix[-1] + 1] if len(ix) else v[:0]
            else:
                sh[k] = v
        out.append(sh)
    return out


def _reduce_results(results):
    """Per-learner metrics -> one dict: per-row arrays concatenated in rank order,
    numbers averaged, anything else from rank 0."""
    if not results:
        return {}
    if not isinstance(results[0], dict):
        return results[0]
    out = {}
    for k, v in results[0].items():
        vals = [r.get(k) for r in results]
        if all(isinstance(x, np.ndarray) for x in vals):
            out[k] = np.concatenate(vals)
        elif all(isinstance(x, (int, float, np.floating, np.integer)) for x in vals):
            out[k] = float(np.mean(vals))
        else:
            out[k] = v
    return out


def _learner_update(kind, batches):
    b = concat_batches(batches) if isinstance(batches, list) else batches
    return _LEARNER.update_ppo(b) if kind == "ppo" else _LEARNER.update_vtrace(b)


def _learner_update_modules(kind, per_module):
    lrs = _LEARNER._module_learners()
    return {m: (lrs[m].update_ppo(b) if kind == "ppo" else lrs[m].update_vtrace(b))
            for m, b in sorted(per_module.items(), key=lambda kv: str(kv[0]))}


def _learner_update_refs(kind, refs):
    import ray_amd as ray

    batches = ray.get(list(refs))  # this learner's fragments, zero-copy from the store
    b = concat_batches(batches) if len(batches) > 1 else batches[0]
    return _LEARNER.update_ppo(b) if kind == "ppo" else _LEARNER.update_vtrace(b)


def _learner_call(name, *a):
    return getattr(_LEARNER, name)(*a)


def _split_b(batch, n, i):
    out = {}
    for k, v in batch.items():
        if isinstance(v, np.ndarray):
            axis = 0 if k in _AXIS0 else 1
            out[k] = np.array_split(v, n, axis=axis)[i]
        else:
            out[k] = v
    return out


class MultiAgentLearnerGroup:
    """The learners of a multi-agent algorithm (reference: rllib/core/learner/
    learner_group.py over a MultiRLModule): ONE LearnerGroup whose every learner holds every
    module — the first module is each learner's own, the others join through
    ``Learner.add_module`` (their own networks, optimizers and losses; gradients averaged
    over the group per module). Runner outputs are split by module id; only the
    ``trainable`` modules are updated."""

    def __init__(self, config: dict, specs: dict, policies_to_train=None):
        self.config = config
        self.specs = dict(specs)
        self.trainable = set(policies_to_train) if policies_to_train else set(specs)
        ids = list(specs)
        self.primary = ids[0]
        self.group = LearnerGroup(config, *specs[self.primary], module_id=self.primary)
        self._hidden = set()  # a removed primary: kept inside the learners, never reported
        for mid in ids[1:]:
            self.group.add_module(module_id=mid, module_spec=tuple(specs[mid]))

    @property
    def module_ids(self) -> list:
        return [m for m in self.specs if m not in self._hidden]

    def _set_trainable(self, spec):
        ids = self.module_ids
        self.trainable = ({m for m in ids if spec(m)} if callable(spec)
                          else set(spec) & set(ids))

    # reference-named module-set API (learner_group.py:494 add_module, :520 remove_module)
    def add_module(self, *, module_id, module_spec, config_overrides=None,
                   new_should_module_be_updated=None):
        spec = tuple(module_spec) if isinstance(module_spec, (tuple, list)) else module_spec
        self.group.add_module(module_id=module_id, module_spec=spec,
                              config_overrides=config_overrides)
        self.specs = dict(self.specs)
        self.specs[module_id] = spec if isinstance(spec, tuple) else \
            (spec.observation_space, spec.action_space)
        if new_should_module_be_updated is None:
            self.trainable.add(module_id)
        else:
            self._set_trainable(new_should_module_be_updated)
        return self.module_ids

    def remove_module(self, module_id, *, new_should_module_be_updated=None):
        if module_id == self.primary:
            self._hidden.add(module_id)  # the learners' own module stays built, unused
        else:
            self.group.remove_module(module_id)
        self.specs = {k: v for k, v in self.specs.items() if k != module_id}
        self.trainable.discard(module_id)
        if new_should_module_be_updated is not None:
            self._set_trainable(new_should_module_be_updated)
        return self.module_ids

    def add(self, mid, spec, trainable=True):
        """Algorithm.add_module's spelling (a trainable flag instead of the update set)."""
        self.add_module(module_id=mid, module_spec=spec)
        if not trainable:
            self.trainable.discard(mid)

    def remove(self, mid):
        self.remove_module(mid)

    def get_module_state(self, module_ids=None) -> dict:
        ids = self.module_ids if module_ids is None else \
            [m for m in module_ids if m in self.module_ids]
        return self.group.get_module_state(ids)

    def set_module_state(self, state: dict):
        self.group.set_module_state(state)

    def get_optimizer_state(self) -> dict:
        return {m: st for m, st in self.group.get_optimizer_state().items()
                if m not in self._hidden}

    def set_optimizer_state(self, state: dict):
        self.group.set_optimizer_state(state)

    def foreach_learner(self, func, **kwargs):
        """{module_id: [func(that module's learner) on every rank]}."""
        out = {}
        for mid in self.module_ids:
            out[mid] = self.group.foreach_learner(_on_module, _mid=mid, _func=func, **kwargs)
        return out

    def update(self, kind, batches):
        per = {}
        for mid in self.module_ids:
            if mid not in self.trainable:
                continue
            mb = [b["modules"][mid] for b in batches if mid in b["modules"]]
            if mb:
                per[mid] = mb
        return self.group.update_modules(kind, per) if per else {}

    def get_weights(self):
        return self.get_module_state()

    def set_weights(self, w):
        self.set_module_state({m: wm for m, wm in w.items() if m in self.specs})

    def get_state(self):
        return {"modules": self.module_ids, "trainable": sorted(self.trainable, key=str),
                "learner": self.group.get_state()}

    def set_state(self, s):
        self.group.set_state(s["learner"])
        self.trainable = set(s.get("trainable") or self.trainable)

    def shutdown(self):
        self.group.shutdown()


def _on_module(lr, _mid, _func, **kwargs):
    return _func(lr._module_learners()[_mid], **kwargs)
