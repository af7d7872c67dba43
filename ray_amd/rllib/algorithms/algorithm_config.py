"""AlgorithmConfig builder (reference: rllib/algorithms/algorithm_config.py)."""

from __future__ import annotations

import copy


class AlgorithmConfig:

    @staticmethod
    def DEFAULT_POLICY_MAPPING_FN(agent_id, episode=None, worker=None, **kwargs):
        """Every agent to the default module (reference: the same static method)."""
        return "default_policy"

    @staticmethod
    def DEFAULT_AGENT_TO_MODULE_MAPPING_FN(agent_id, episode=None):
        return "default_policy"


    algo_class = None

    def __init__(self, algo_class=None):
        self.algo_class = algo_class or type(self).algo_class
        self.env = None
        self.env_config = {}
        self.num_env_runners = 2
        self.num_envs_per_env_runner = 1
        self.rollout_fragment_length = 200
        self.num_cpus_per_env_runner = 1
        self.num_gpus_per_env_runner = 0
        # > 0: the runners' policy forward runs batched in ONE GPU process holding this GPU
        # share (rllib/env/policy_server.py); the runners keep stepping envs on CPU
        self.num_gpus_per_policy_server = 0
        self.gamma = 0.99
        self.lr = 5e-5
        self.train_batch_size = 4000
        self.model = {}
        self.grad_clip = None
        self.num_learners = 0
        self.num_gpus_per_learner = 1
        self.seed = None
        self.evaluation_interval = None
        self.evaluation_duration = 10
        self.evaluation_num_env_runners = 0
        self.evaluation_config = {}
        self.min_time_s_per_iteration = None
        self.framework_str = "torch"
        self.learner_bf16 = True
        self.bootstrap_truncated = False
        self.metrics_num_episodes_for_smoothing = 100
        self.input_ = None
        self.output = None
        self.policies = None
        self.policy_mapping_fn = None
        self.policies_to_train = None
        # ConnectorV2 pipelines (callables returning connector(s)) and observation filter
        self.env_to_module_connector = None
        self.module_to_env_connector = None
        self.learner_connector = None
        self.observation_filter = "NoFilter"
        # sample the next train batch while the learner updates on this one (one
        # iteration of policy lag; the PPO ratio uses the recorded behaviour logp)
        self.sample_async = False
        self.callbacks_class = None
        # RLModule / Learner extensibility (reference: AlgorithmConfig.rl_module, training
        # learner_class)
        self._rl_module_spec = None
        self.learner_class = None
        # fault tolerance (reference: AlgorithmConfig.fault_tolerance, algorithm_config.py
        # :2673): recreate dead EnvRunners and resync their weights
        self.restart_failed_env_runners = True
        self.ignore_env_runner_failures = False
        self.max_num_env_runner_restarts = 1000
        self.delay_between_env_runner_restarts_s = 0.0
        self.env_runner_health_probe_timeout_s = 30.0
        self.restart_failed_sub_environments = False
        self.evaluation_parallel_to_training = False
        self.evaluation_duration_unit = "episodes"
        self.checkpoint_trainable_policies_only = False
        self.explore = True
        self.exploration_config = {}
        self.keep_per_episode_custom_metrics = False
        self.extra_python_environs_for_driver = {}
        self.extra_python_environs_for_worker = {}
        # environment() (reference: algorithm_config.py:1385-1398): rewards clipped in the
        # train batch (True: sign, float c: [-c, c]); Box actions unsquashed from [-1, 1]
        # to the bounds (normalize_actions) or clipped to them (clip_actions)
        self.clip_rewards = None
        self.normalize_actions = True
        self.clip_actions = False
        self.observation_space = None
        self.action_space = None
        self.render_env = False
        self.disable_env_checking = False
        self.action_mask_key = "action_mask"
        self.env_task_fn = None
        # env_runners() (reference: :1515 batch_mode and the runner options around it)
        self.batch_mode = "truncate_episodes"
        self.sample_timeout_s = 60.0
        self.create_env_on_local_worker = False
        self.custom_resources_per_env_runner = {}
        self.validate_env_runners_after_construction = True
        self.max_requests_in_flight_per_env_runner = 2
        self.episode_lookback_horizon = 1
        self.compress_observations = False
        self.remote_worker_envs = False
        self.remote_env_batch_wait_ms = 0
        self.add_default_connectors_to_env_to_module_pipeline = True
        self.add_default_connectors_to_module_to_env_pipeline = True
        self.update_worker_filter_stats = True
        self.use_worker_filter_stats = True
        # evaluation(): off-policy estimation on logged data (reference: :2040)
        self.off_policy_estimation_methods = {}
        self.ope_split_batch_by_episode = True
        # offline_data() readers / writers (reference: :2379)
        self.input_read_method = None
        self.input_read_method_kwargs = None
        self.output_write_method = "write_json"
        self.output_max_rows_per_file = 100_000
        self.shuffle_buffer_size = None
        # learners()
        self.num_cpus_per_learner = 1
        self.local_gpu_idx = 0
        # checkpointing() / debugging() / reporting()
        self.export_native_model_files = False
        self.log_level = "WARN"
        self.log_sys_usage = True
        self.logger_config = None
        self.fake_sampler = False
        self.keep_per_episode_custom_metrics = False
        self.min_sample_timesteps_per_iteration = 0
        self.min_train_timesteps_per_iteration = 0

    # ---------------------------------------------------------------- builders
    def _set_keys(self, method: str, kw: dict, known, renames=None) -> "AlgorithmConfig":
        """Set builder keywords: every key must be one this builder knows (a typo raises
        instead of being silently dropped); None leaves the current value."""
        renames = renames or {}
        unknown = sorted(k for k in kw if k not in known and k not in renames)
        if unknown:
            raise ValueError(f"{type(self).__name__}.{method}() got unknown key(s) {unknown}")
        for k, v in kw.items():
            if v is not None:
                setattr(self, renames.get(k, k), v)
        return self

    _ENV_KEYS = ("observation_space", "action_space", "render_env", "clip_rewards",
                 "normalize_actions", "clip_actions", "disable_env_checking",
                 "action_mask_key", "env_task_fn")

    def environment(self, env=None, *, env_config=None, is_atari=None, **kw):
        """reference: AlgorithmConfig.environment (algorithm_config.py:1360)."""
        if env is not None:
            self.env = env
        if env_config is not None:
            self.env_config = dict(env_config)
        if is_atari is not None:
            self._is_atari = bool(is_atari)
        if kw.get("clip_rewards") not in (None, True, False) and \
                not isinstance(kw["clip_rewards"], (int, float)):
            raise ValueError("clip_rewards must be None, a bool or a float bound")
        return self._set_keys("environment", kw, self._ENV_KEYS)

    _RUNNER_KEYS = ("num_env_runners", "num_envs_per_env_runner", "rollout_fragment_length",
                    "num_cpus_per_env_runner", "num_gpus_per_env_runner",
                    "num_gpus_per_policy_server", "env_to_module_connector", "module_to_env_connector",
                    "observation_filter", "sample_async", "batch_mode", "explore",
                    "exploration_config", "sample_timeout_s", "create_env_on_local_worker",
                    "custom_resources_per_env_runner", "validate_env_runners_after_construction",
                    "max_requests_in_flight_per_env_runner", "episode_lookback_horizon",
                    "compress_observations", "remote_worker_envs", "remote_env_batch_wait_ms",
                    "add_default_connectors_to_env_to_module_pipeline",
                    "add_default_connectors_to_module_to_env_pipeline",
                    "update_worker_filter_stats", "use_worker_filter_stats")

    def env_runners(self, **kw):
        """reference: AlgorithmConfig.env_runners (algorithm_config.py:1480)."""
        bm = kw.get("batch_mode")
        if bm is not None and bm not in ("truncate_episodes", "complete_episodes"):
            raise ValueError(f"batch_mode must be 'truncate_episodes' or 'complete_episodes', "
                             f"got {bm!r}")
        return self._set_keys("env_runners", kw, self._RUNNER_KEYS,
                              {"create_local_env_runner": "create_env_on_local_worker",
                               "num_rollout_workers": "num_env_runners",
                               "num_envs_per_worker": "num_envs_per_env_runner"})

    def rollouts(self, *, num_rollout_workers=None, num_envs_per_worker=None, **kw):
        return self.env_runners(num_env_runners=num_rollout_workers,
                                num_envs_per_env_runner=num_envs_per_worker, **kw)

    # training() keys the learners read without a config default (RLlib options of this
    # framework: the learner group's collective backend, HIP-graph capture of the learner
    # update, bf16 CPU inference in env runners, per-learner batch)
    _TRAINING_EXTRA = frozenset({"learner_backend", "learner_cuda_graph", "env_runner_bf16",
                                 "train_batch_size_per_learner", "learner_class", "model",
                                 "optimizer", "grad_clip_by"})

    def training(self, **kw):
        """Set training hyperparameters. Keys must be known to this algorithm's config
        (its defaults, the reference's old names, or _TRAINING_EXTRA): a typo raises instead
        of being silently ignored."""
        aliases = {"sgd_minibatch_size": "minibatch_size", "num_sgd_iter": "num_epochs",
                   "lambda": "lambda_"}
        known = set(vars(self)) | self._TRAINING_EXTRA
        unknown = sorted(k for k in kw if aliases.get(k, k) not in known)
        if unknown:
            raise ValueError(f"{type(self).__name__}.training() got unknown key(s) {unknown}")
        for k, v in kw.items():
            if v is None:
                continue
            setattr(self, aliases.get(k, k), v)
        return self

    def resources(self, *, num_gpus=None, num_cpus_for_main_process=None,
                  num_cpus_per_worker=None, num_gpus_per_worker=None, **kw):
        self._set_keys("resources", kw, ("placement_strategy", "custom_resources_per_worker",
                                         "num_cpus_per_learner_worker",
                                         "num_gpus_per_learner_worker", "num_learner_workers"),
                       )
        if num_gpus is not None:
            self.num_gpus_per_learner = num_gpus if num_gpus <= 1 else 1
            if num_gpus > 1:
                self.num_learners = int(num_gpus)
        if num_cpus_for_main_process is not None:
            self.num_cpus_for_main_process = num_cpus_for_main_process
        if num_cpus_per_worker is not None:
            self.num_cpus_per_env_runner = num_cpus_per_worker
        if num_gpus_per_worker is not None:
            self.num_gpus_per_env_runner = num_gpus_per_worker
        return self

    def learners(self, **kw):
        """reference: AlgorithmConfig.learners (algorithm_config.py:2200)."""
        return self._set_keys("learners", kw, ("num_learners", "num_gpus_per_learner",
                                               "num_cpus_per_learner", "local_gpu_idx",
                                               "max_requests_in_flight_per_learner"))

    def callbacks(self, callbacks_class=None, **kw):
        """RLlibCallback subclass / instance / list of them (reference:
        AlgorithmConfig.callbacks); per-event callables (``on_episode_end=fn``, ...) are
        kept in ``callbacks_on_events``."""
        if kw:
            events = ("on_algorithm_init", "on_train_result", "on_evaluate_start",
                      "on_evaluate_end", "on_env_runners_recreated", "on_checkpoint_loaded",
                      "on_environment_created", "on_episode_created", "on_episode_start",
                      "on_episode_step", "on_episode_end", "on_sample_end")
            bad = sorted(k for k in kw if k not in events)
            if bad:
                raise ValueError(f"{type(self).__name__}.callbacks() got unknown key(s) {bad}")
            self.callbacks_on_events = {k: v for k, v in kw.items() if v is not None}
        self.callbacks_class = callbacks_class
        return self

    def rl_module(self, *, rl_module_spec=None, model_config=None, model_config_dict=None,
                  algorithm_config_overrides_per_module=None, **kw):
        """A user RLModule (RLModuleSpec / MultiRLModuleSpec) and / or the model config
        of the default modules (reference: AlgorithmConfig.rl_module)."""
        if kw:
            raise ValueError(f"{type(self).__name__}.rl_module() got unknown key(s) "
                             f"{sorted(kw)}")
        if algorithm_config_overrides_per_module is not None:
            self.algorithm_config_overrides_per_module = dict(
                algorithm_config_overrides_per_module)
        if rl_module_spec is not None:
            self._rl_module_spec = rl_module_spec
        mc = model_config if model_config is not None else model_config_dict
        if mc is not None:
            self.model = dict(getattr(mc, "__dict__", mc)) if not isinstance(mc, dict) \
                else dict(mc)
        return self

    @property
    def rl_module_spec(self):
        return self._rl_module_spec

    @property
    def model_config(self):
        return dict(self.model or {})

    def get_rl_module_spec(self, env=None, spaces=None):
        from ray_amd.rllib.core.rl_module import RLModuleSpec

        return self._rl_module_spec or RLModuleSpec(model_config=dict(self.model or {}))

    def get_default_learner_class(self):
        from ray_amd.rllib.core.learner import Learner

        return Learner

    def fault_tolerance(self, *, restart_failed_env_runners=None,
                        ignore_env_runner_failures=None, max_num_env_runner_restarts=None,
                        delay_between_env_runner_restarts_s=None,
                        env_runner_health_probe_timeout_s=None,
                        restart_failed_sub_environments=None, recreate_failed_env_runners=None,
                        **kw):
        self._set_keys("fault_tolerance", kw, ("num_consecutive_env_runner_failures_tolerance",
                                               "env_runner_restore_timeout_s"))
        if recreate_failed_env_runners is not None:  # old name
            restart_failed_env_runners = recreate_failed_env_runners
        for k, v in dict(restart_failed_env_runners=restart_failed_env_runners,
                         ignore_env_runner_failures=ignore_env_runner_failures,
                         max_num_env_runner_restarts=max_num_env_runner_restarts,
                         delay_between_env_runner_restarts_s=delay_between_env_runner_restarts_s,
                         env_runner_health_probe_timeout_s=env_runner_health_probe_timeout_s,
                         restart_failed_sub_environments=restart_failed_sub_environments
                         ).items():
            if v is not None:
                setattr(self, k, v)
        return self

    def checkpointing(self, **kw):
        return self._set_keys("checkpointing", kw, ("export_native_model_files",
                                                    "checkpoint_trainable_policies_only"))

    def exploration(self, *, explore=None, exploration_config=None, **kw):
        if kw:
            raise ValueError(f"{type(self).__name__}.exploration() got unknown key(s) "
                             f"{sorted(kw)}")
        if explore is not None:
            self.explore = bool(explore)
        if exploration_config is not None:
            self.exploration_config = dict(exploration_config)
        return self

    def python_environment(self, *, extra_python_environs_for_driver=None,
                           extra_python_environs_for_worker=None, **kw):
        if kw:
            raise ValueError(f"{type(self).__name__}.python_environment() got unknown "
                             f"key(s) {sorted(kw)}")
        if extra_python_environs_for_driver is not None:
            self.extra_python_environs_for_driver = dict(extra_python_environs_for_driver)
        if extra_python_environs_for_worker is not None:
            self.extra_python_environs_for_worker = dict(extra_python_environs_for_worker)
        return self

    def experimental(self, **kw):
        known = ("_validate_config", "_use_msgpack_checkpoints", "_torch_grad_scaler_class",
                 "_torch_lr_scheduler_classes", "_tf_policy_handles_more_than_one_loss",
                 "_disable_preprocessor_api", "_disable_action_flattening",
                 "_disable_initialize_loss_from_dummy_batch", "_disable_execution_plan_api",
                 "_enable_new_api_stack")
        bad = sorted(k for k in kw if k not in known and "_" + k not in known)
        if bad:
            raise ValueError(f"{type(self).__name__}.experimental() got unknown key(s) {bad}")
        for k, v in kw.items():
            setattr(self, k.lstrip("_"), v)
        return self

    def validate(self):
        if self.num_env_runners < 0:
            raise ValueError("num_env_runners must be >= 0")
        if self.evaluation_num_env_runners < 0:
            raise ValueError("evaluation_num_env_runners must be >= 0")
        if isinstance(self.train_batch_size, int) and self.train_batch_size <= 0:
            raise ValueError("train_batch_size must be > 0")
        return True

    def freeze(self):
        """After this, setting any attribute raises (reference: AlgorithmConfig.freeze —
        the Algorithm freezes its copy so a running algorithm's config cannot drift)."""
        object.__setattr__(self, "_is_frozen", True)
        return self

    def __setattr__(self, k, v):
        if self.__dict__.get("_is_frozen", False):
            raise AttributeError(f"Cannot set attribute ({k}) of an already frozen "
                                 "AlgorithmConfig; use config.copy(copy_frozen=False)")
        object.__setattr__(self, k, v)

    # ---------------------------------------------------------------- dict-like access
    def keys(self):
        return self.to_dict().keys()

    def values(self):
        return self.to_dict().values()

    def items(self):
        return self.to_dict().items()

    def pop(self, k, default=None):
        if self.__dict__.get("_is_frozen", False):
            raise AttributeError("Cannot pop from a frozen AlgorithmConfig")
        return self.__dict__.pop(k, default)

    # ---------------------------------------------------------------- derived settings
    @property
    def num_workers(self):  # old name of num_env_runners
        return self.num_env_runners

    @property
    def uses_new_env_runners(self):
        return True

    @property
    def is_atari(self) -> bool:
        if self.__dict__.get("_is_atari") is not None:
            return self.__dict__["_is_atari"]
        e = self.env if isinstance(self.env, str) else ""
        return e.startswith("ALE/") or "NoFrameskip" in e

    @property
    def total_train_batch_size(self) -> int:
        """train_batch_size_per_learner x max(1, num_learners) when set per learner, else
        train_batch_size (reference: AlgorithmConfig.total_train_batch_size)."""
        per = getattr(self, "train_batch_size_per_learner", None)
        if per:
            return int(per) * max(1, int(self.num_learners or 0))
        return int(self.train_batch_size)

    def get_rollout_fragment_length(self, worker_index: int = 0) -> int:
        """'auto' = the train batch split evenly over all env-runner envs (worker_index
        1..N gets one extra step while the split has a remainder)."""
        if self.rollout_fragment_length != "auto":
            return int(self.rollout_fragment_length)
        nr = max(1, self.num_env_runners)
        per_env = self.total_train_batch_size // (nr * self.num_envs_per_env_runner)
        rem = self.total_train_batch_size - per_env * nr * self.num_envs_per_env_runner
        extra = 1 if worker_index and rem and worker_index * self.num_envs_per_env_runner <= rem \
            else 0
        return max(1, per_env + extra)

    def validate_train_batch_size_vs_rollout_fragment_length(self):
        """The sampled fragments must be able to fill one train batch within 10 % (the
        reference's tolerance); otherwise raise with the rollout_fragment_length to use."""
        if self.rollout_fragment_length == "auto":
            return
        per_round = max(1, self.num_env_runners) * self.num_envs_per_env_runner * \
            int(self.rollout_fragment_length)
        tb = self.total_train_batch_size
        if per_round > tb and per_round - tb > 0.1 * tb:
            suggested = max(1, tb // (max(1, self.num_env_runners) *
                                      self.num_envs_per_env_runner))
            raise ValueError(
                f"one sampling round ({per_round} env steps = num_env_runners x "
                f"num_envs_per_env_runner x rollout_fragment_length) exceeds the train batch "
                f"({tb}) by more than 10%; set rollout_fragment_length={suggested} or 'auto'")

    @property
    def multiagent(self) -> dict:
        return {"policies": self.policies, "policy_mapping_fn": self.policy_mapping_fn,
                "policies_to_train": self.policies_to_train}

    def get_multi_agent_setup(self, *, env=None, spaces=None, default_policy_class=None):
        """(policies dict id -> (obs_space, act_space), policy_mapping_fn). Module ids
        given without spaces take the env's single-agent spaces."""
        if self.policies is None:
            from ray_amd.rllib.core.learner import DEFAULT_MODULE_ID

            pol = {DEFAULT_MODULE_ID: None}
        elif isinstance(self.policies, dict):
            pol = dict(self.policies)
        else:
            pol = {pid: None for pid in self.policies}
        if any(v is None for v in pol.values()):
            obs, act = (spaces or (None, None))
            if obs is None and (env is not None or self.env is not None):
                from ray_amd.rllib.env.envs import make_env

                e = env if env is not None else make_env(self.env, self.env_config)
                obs, act = e.observation_space, e.action_space
            pol = {k: (v if v is not None else (obs, act)) for k, v in pol.items()}
        fn = self.policy_mapping_fn or (lambda agent_id, *a, **k: next(iter(pol)))
        return pol, fn

    def get_config_for_module(self, module_id):
        """This config with the per-module overrides applied (reference:
        AlgorithmConfig.get_config_for_module; overrides come from
        ``algorithm_config_overrides_per_module={module_id: {key: value}}`` passed to
        multi_agent())."""
        ov = (getattr(self, "algorithm_config_overrides_per_module", None) or {}).get(module_id)
        if not ov:
            return self
        c = self.copy(copy_frozen=False)
        c.update_from_dict(dict(ov))
        return c

    def get_evaluation_config_object(self):
        """A copy of this config with ``evaluation_config`` applied on top, evaluation of
        the evaluation config disabled (what the evaluation EnvRunners are built from)."""
        c = self.copy(copy_frozen=False)
        c.update_from_dict(dict(self.evaluation_config or {}))
        c.evaluation_interval = None
        c.num_env_runners = self.evaluation_num_env_runners
        if "explore" not in (self.evaluation_config or {}):
            c.explore = False
        return c

    def get_default_rl_module_spec(self):
        from ray_amd.rllib.core.rl_module import RLModuleSpec

        return RLModuleSpec(model_config=dict(self.model or {}))

    def get_marl_module_spec(self, *, env=None, spaces=None):
        """MultiRLModuleSpec over get_multi_agent_setup's modules."""
        from ray_amd.rllib.core.rl_module import MultiRLModuleSpec, RLModuleSpec

        if isinstance(self._rl_module_spec, MultiRLModuleSpec):
            return self._rl_module_spec
        pol, _ = self.get_multi_agent_setup(env=env, spaces=spaces)
        base = self._rl_module_spec
        specs = {}
        for mid, sp in pol.items():
            obs, act = sp if isinstance(sp, tuple) else (None, None)
            specs[mid] = RLModuleSpec(
                module_class=getattr(base, "module_class", None), observation_space=obs,
                action_space=act, model_config=dict(getattr(base, "model_config", None)
                                                    or self.model or {}))
        return MultiRLModuleSpec(rl_module_specs=specs)

    def get_torch_compile_worker_config(self) -> dict:
        """No torch.compile on this stack: the MI355X learner's hot path is hand-written HIP
        kernels replayed as HIP graphs, so there is nothing to configure."""
        return {"torch_compile": False}

    # ---------------------------------------------------------------- builders of parts
    def build_env_to_module_connector(self, env=None, spaces=None):
        from ray_amd.rllib.connectors.connector_v2 import build_pipeline

        obs, act = self._spaces(env, spaces)
        return build_pipeline(self.env_to_module_connector, obs, act)

    def build_module_to_env_connector(self, env=None, spaces=None):
        from ray_amd.rllib.connectors.connector_v2 import build_pipeline

        obs, act = self._spaces(env, spaces)
        return build_pipeline(self.module_to_env_connector, obs, act)

    def build_learner_connector(self, input_observation_space=None,
                                input_action_space=None, device=None):
        from ray_amd.rllib.connectors.connector_v2 import build_pipeline

        return build_pipeline(self.learner_connector, input_observation_space,
                              input_action_space)

    def _spaces(self, env, spaces):
        if spaces is not None:
            return spaces
        from ray_amd.rllib.env.envs import make_env

        e = env if env is not None else make_env(self.env, self.env_config)
        return e.observation_space, e.action_space

    def build_learner_group(self, *, env=None, spaces=None):
        """The LearnerGroup an Algorithm of this config trains with (num_learners remote
        learner actors over RCCL/gloo, or one local learner)."""
        from ray_amd.rllib.core.learner import LearnerGroup

        obs, act = self._spaces(env, spaces)
        cfg = self.to_dict()
        cfg.setdefault("module_kind", "actor_critic")
        return LearnerGroup(cfg, obs, act)

    def build_learner(self, *, env=None, spaces=None, device=None):
        """One local Learner (the configured learner_class, default per algorithm)."""
        from ray_amd.rllib.core.learner import _learner_cls

        obs, act = self._spaces(env, spaces)
        cfg = self.to_dict()
        cfg.setdefault("module_kind", "actor_critic")
        return _learner_cls(cfg)(cfg, obs, act, device=device)

    def serialize(self) -> dict:
        """JSON-able dict: classes and callables as their qualified names."""
        def conv(v):
            if isinstance(v, (str, int, float, bool)) or v is None:
                return v
            if isinstance(v, dict):
                return {str(k): conv(x) for k, x in v.items()}
            if isinstance(v, (list, tuple, set)):
                return [conv(x) for x in v]
            if isinstance(v, type) or callable(v):
                return f"{getattr(v, '__module__', '?')}.{getattr(v, '__qualname__', repr(v))}"
            return repr(v)

        return {k: conv(v) for k, v in self.to_dict().items() if k != "_is_frozen"}

    @classmethod
    def overrides(cls, **kwargs) -> dict:
        """Validated per-module / evaluation override dict (reference:
        AlgorithmConfig.overrides): unknown keys raise."""
        proto = cls()
        for k in kwargs:
            if not hasattr(proto, cls._LEGACY_KEYS.get(k, k)):
                raise KeyError(f"unknown AlgorithmConfig key in overrides: {k}")
        return dict(kwargs)

    @classmethod
    def from_dict(cls, d: dict):
        return cls().update_from_dict(d)

    def framework(self, framework="torch", **kw):
        # tf / torch.compile options of the reference: accepted and recorded; this stack
        # has no tracing compiler (HIP graphs + hand-written kernels)
        self._set_keys("framework", kw, (
            "eager_tracing", "eager_max_retraces", "tf_session_args", "local_tf_session_args",
            "torch_compile_learner", "torch_compile_learner_what_to_compile",
            "torch_compile_learner_dynamo_mode", "torch_compile_learner_dynamo_backend",
            "torch_compile_worker", "torch_compile_worker_dynamo_backend",
            "torch_compile_worker_dynamo_mode", "torch_ddp_kwargs",
            "torch_skip_nan_gradients"))
        if framework not in ("torch",):
            raise ValueError("ray_amd RLlib supports framework='torch' only (MI355X/ROCm)")
        self.framework_str = framework
        return self

    def debugging(self, **kw):
        return self._set_keys("debugging", kw, ("seed", "log_level", "log_sys_usage",
                                                "logger_config", "fake_sampler",
                                                "logger_creator"))

    _EVAL_KEYS = ("evaluation_sample_timeout_s", "evaluation_force_reset_envs_before_iteration",
                  "evaluation_auto_duration_min_env_steps_per_sample",
                  "evaluation_auto_duration_max_env_steps_per_sample", "custom_evaluation_function",
                  "off_policy_estimation_methods", "ope_split_batch_by_episode",
                  "always_attach_evaluation_results")

    def evaluation(self, *, evaluation_interval=None, evaluation_duration=None,
                   evaluation_num_env_runners=None, evaluation_config=None,
                   evaluation_parallel_to_training=None, evaluation_duration_unit=None,
                   evaluation_num_workers=None, **kw):
        if evaluation_num_workers is not None:  # old name
            evaluation_num_env_runners = evaluation_num_workers
        self._set_keys("evaluation", kw, self._EVAL_KEYS)
        if evaluation_parallel_to_training is not None:
            self.evaluation_parallel_to_training = bool(evaluation_parallel_to_training)
        if evaluation_duration_unit is not None:
            if evaluation_duration_unit not in ("episodes", "timesteps"):
                raise ValueError("evaluation_duration_unit must be 'episodes' or 'timesteps'")
            self.evaluation_duration_unit = evaluation_duration_unit
        if evaluation_interval is not None:
            self.evaluation_interval = evaluation_interval
        if evaluation_duration is not None:
            self.evaluation_duration = evaluation_duration
        if evaluation_num_env_runners is not None:
            self.evaluation_num_env_runners = evaluation_num_env_runners
        if evaluation_config is not None:
            self.evaluation_config = evaluation_config
        return self

    def reporting(self, *, min_time_s_per_iteration=None, metrics_num_episodes_for_smoothing=None,
                  **kw):
        self._set_keys("reporting", kw, ("keep_per_episode_custom_metrics",
                                         "min_sample_timesteps_per_iteration",
                                         "min_train_timesteps_per_iteration",
                                         "metrics_episode_collection_timeout_s", "log_gradients"))
        if min_time_s_per_iteration is not None:
            self.min_time_s_per_iteration = min_time_s_per_iteration
        if metrics_num_episodes_for_smoothing is not None:
            self.metrics_num_episodes_for_smoothing = metrics_num_episodes_for_smoothing
        return self

    _OFFLINE_KEYS = ("input_config", "input_read_method", "input_read_method_kwargs",
                     "input_read_schema", "input_read_episodes", "input_read_sample_batches",
                     "input_read_batch_size", "input_filesystem", "input_compress_columns",
                     "map_batches_kwargs", "iter_batches_kwargs", "prelearner_class",
                     "dataset_num_iters_per_learner", "actions_in_input_normalized",
                     "postprocess_inputs", "shuffle_buffer_size", "output_config",
                     "output_compress_columns", "output_max_file_size",
                     "output_max_rows_per_file", "output_write_method",
                     "output_write_episodes", "offline_sampling")

    def offline_data(self, *, input_=None, output=None, **kw):
        """Offline experience source / sink (reference: AlgorithmConfig.offline_data,
        algorithm_config.py:2379): ``input_`` is a path / list of paths (JSON lines or
        parquet, read through ray_amd.data) or "sampler"."""
        self._set_keys("offline_data", kw, self._OFFLINE_KEYS)
        if input_ is not None:
            self.input_ = input_
        if output is not None:
            self.output = output
        return self

    def multi_agent(self, *, policies=None, policy_mapping_fn=None, policies_to_train=None,
                    algorithm_config_overrides_per_module=None, **kw):
        """reference: AlgorithmConfig.multi_agent -- ``policies`` is a set/list of module ids
        or a dict id -> (observation_space, action_space) / PolicySpec / None."""
        self._set_keys("multi_agent", kw, ("policy_map_capacity", "policy_states_are_swappable",
                                           "observation_fn", "count_steps_by"))
        if policies is not None:
            self.policies = policies
        if policy_mapping_fn is not None:
            self.policy_mapping_fn = policy_mapping_fn
        if policies_to_train is not None:
            self.policies_to_train = list(policies_to_train)
        if algorithm_config_overrides_per_module is not None:
            self.algorithm_config_overrides_per_module = dict(
                algorithm_config_overrides_per_module)
        return self

    @property
    def is_multi_agent(self):
        return self.policies is not None

    def api_stack(self, **kw):
        return self._set_keys("api_stack", kw, ("enable_rl_module_and_learner",
                                                "enable_env_runner_and_connector_v2"))

    # old-API-stack config keys (tuned-example YAML files) -> current attribute names
    _LEGACY_KEYS = {"lambda": "lambda_", "num_workers": "num_env_runners",
                    "num_rollout_workers": "num_env_runners",
                    "num_envs_per_worker": "num_envs_per_env_runner",
                    "num_sgd_iter": "num_epochs", "sgd_minibatch_size": "minibatch_size",
                    "framework": "framework_str", "callbacks": "callbacks_class",
                    "num_cpus_per_worker": "num_cpus_per_env_runner",
                    "num_gpus_per_worker": "num_gpus_per_env_runner"}

    def update_from_dict(self, d: dict):
        for k, v in d.items():
            if k == "num_gpus":
                self.resources(num_gpus=v)
                continue
            name = self._LEGACY_KEYS.get(k, k)
            prop = getattr(type(self), name, None)
            if isinstance(prop, property) and prop.fset is None:
                continue  # derived (is_multi_agent, model_config, ...): not settable
            setattr(self, name, v)
        return self

    def copy(self, copy_frozen=None):
        c = copy.deepcopy(self)
        if not copy_frozen:  # None / False: the copy is writable (reference default)
            c.__dict__.pop("_is_frozen", None)
        return c

    def to_dict(self) -> dict:
        return {k: v for k, v in self.__dict__.items() if k not in ("algo_class", "_is_frozen")}

    def get(self, k, default=None):
        return getattr(self, k, default)

    def __getitem__(self, k):
        return getattr(self, k)

    def build(self, env=None, logger_creator=None):
        if env is not None:
            self.env = env
        if self.algo_class is None:
            raise ValueError("no algorithm class bound to this config")
        return self.algo_class(self.copy())

    def build_algo(self, *a, **k):
        return self.build(*a, **k)
