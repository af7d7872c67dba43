"""AlgorithmConfig builder (reference: rllib/algorithms/algorithm_config.py)."""

from __future__ import annotations

import copy


class AlgorithmConfig:
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

    # ---------------------------------------------------------------- builders
    def environment(self, env=None, *, env_config=None, **kw):
        if env is not None:
            self.env = env
        if env_config is not None:
            self.env_config = dict(env_config)
        return self

    def env_runners(self, *, num_env_runners=None, num_envs_per_env_runner=None,
                    rollout_fragment_length=None, num_cpus_per_env_runner=None,
                    num_gpus_per_env_runner=None, env_to_module_connector=None,
                    module_to_env_connector=None, observation_filter=None,
                    sample_async=None, **kw):
        for k, v in dict(num_env_runners=num_env_runners,
                         num_envs_per_env_runner=num_envs_per_env_runner,
                         rollout_fragment_length=rollout_fragment_length,
                         num_cpus_per_env_runner=num_cpus_per_env_runner,
                         num_gpus_per_env_runner=num_gpus_per_env_runner,
                         env_to_module_connector=env_to_module_connector,
                         module_to_env_connector=module_to_env_connector,
                         observation_filter=observation_filter,
                         sample_async=sample_async).items():
            if v is not None:
                setattr(self, k, v)
        return self

    def rollouts(self, *, num_rollout_workers=None, num_envs_per_worker=None, **kw):
        return self.env_runners(num_env_runners=num_rollout_workers,
                                num_envs_per_env_runner=num_envs_per_worker, **kw)

    def training(self, **kw):
        aliases = {"sgd_minibatch_size": "minibatch_size", "num_sgd_iter": "num_epochs",
                   "lambda": "lambda_"}
        for k, v in kw.items():
            if v is None:
                continue
            setattr(self, aliases.get(k, k), v)
        return self

    def resources(self, *, num_gpus=None, **kw):
        if num_gpus is not None:
            self.num_gpus_per_learner = num_gpus if num_gpus <= 1 else 1
            if num_gpus > 1:
                self.num_learners = int(num_gpus)
        return self

    def learners(self, *, num_learners=None, num_gpus_per_learner=None, **kw):
        if num_learners is not None:
            self.num_learners = num_learners
        if num_gpus_per_learner is not None:
            self.num_gpus_per_learner = num_gpus_per_learner
        return self

    def callbacks(self, callbacks_class=None, **kw):
        """RLlibCallback subclass / instance / list of them (reference:
        AlgorithmConfig.callbacks)."""
        self.callbacks_class = callbacks_class
        return self

    def rl_module(self, *, rl_module_spec=None, model_config=None, model_config_dict=None,
                  **kw):
        """A user RLModule (RLModuleSpec / MultiRLModuleSpec) and / or the model config
        of the default modules (reference: AlgorithmConfig.rl_module)."""
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

    def checkpointing(self, *, export_native_model_files=None,
                      checkpoint_trainable_policies_only=None, **kw):
        if checkpoint_trainable_policies_only is not None:
            self.checkpoint_trainable_policies_only = checkpoint_trainable_policies_only
        return self

    def exploration(self, *, explore=None, exploration_config=None, **kw):
        if explore is not None:
            self.explore = bool(explore)
        if exploration_config is not None:
            self.exploration_config = dict(exploration_config)
        return self

    def python_environment(self, *, extra_python_environs_for_driver=None,
                           extra_python_environs_for_worker=None, **kw):
        if extra_python_environs_for_driver is not None:
            self.extra_python_environs_for_driver = dict(extra_python_environs_for_driver)
        if extra_python_environs_for_worker is not None:
            self.extra_python_environs_for_worker = dict(extra_python_environs_for_worker)
        return self

    def experimental(self, **kw):
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
        self._is_frozen = True
        return self

    @classmethod
    def from_dict(cls, d: dict):
        return cls().update_from_dict(d)

    def framework(self, framework="torch", **kw):
        if framework not in ("torch",):
            raise ValueError("ray_amd RLlib supports framework='torch' only (MI355X/ROCm)")
        self.framework_str = framework
        return self

    def debugging(self, *, seed=None, **kw):
        if seed is not None:
            self.seed = seed
        return self

    def evaluation(self, *, evaluation_interval=None, evaluation_duration=None,
                   evaluation_num_env_runners=None, evaluation_config=None,
                   evaluation_parallel_to_training=None, evaluation_duration_unit=None, **kw):
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
        if min_time_s_per_iteration is not None:
            self.min_time_s_per_iteration = min_time_s_per_iteration
        if metrics_num_episodes_for_smoothing is not None:
            self.metrics_num_episodes_for_smoothing = metrics_num_episodes_for_smoothing
        return self

    def offline_data(self, *, input_=None, output=None, **kw):
        """Offline experience source / sink (reference: AlgorithmConfig.offline_data)."""
        if input_ is not None:
            self.input_ = input_
        if output is not None:
            self.output = output
        return self

    def multi_agent(self, *, policies=None, policy_mapping_fn=None, policies_to_train=None,
                    **kw):
        """reference: AlgorithmConfig.multi_agent -- ``policies`` is a set/list of module ids
        or a dict id -> (observation_space, action_space) / PolicySpec / None."""
        if policies is not None:
            self.policies = policies
        if policy_mapping_fn is not None:
            self.policy_mapping_fn = policy_mapping_fn
        if policies_to_train is not None:
            self.policies_to_train = list(policies_to_train)
        return self

    @property
    def is_multi_agent(self):
        return self.policies is not None

    def api_stack(self, **kw):
        return self

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
        return copy.deepcopy(self)

    def to_dict(self) -> dict:
        return {k: v for k, v in self.__dict__.items() if k != "algo_class"}

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
