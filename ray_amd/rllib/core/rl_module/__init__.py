"""RLModules (reference: rllib/core/rl_module/).

``default`` holds the built-in MI355X modules (actor-critic with the HIP conv / fused-head
fast paths, Q-network, SAC actor/critics); ``rl_module`` the user-extensibility layer
(RLModuleSpec, TorchRLModule, stateful modules) and the builder every Learner / EnvRunner
uses. This package's namespace binds no ``torch`` name, so the ``torch`` subpackage
(reference path ``rl_module.torch.TorchRLModule``) can be imported safely."""

from ray_amd.rllib.core.rl_module.default import (MLP, NatureCNN, QModule,  # noqa: F401
                                                  RLModule, SquashedGaussianPolicy, TwinQ,
                                                  gaussian_entropy, gaussian_logp)
from ray_amd.rllib.core.rl_module.rl_module import (MultiRLModuleSpec,  # noqa: F401
                                                    RLModuleSpec, TorchRLModule,
                                                    ValueFunctionAPI, build_module)

from ray_amd.rllib.core.rl_module.checkpoint import MultiRLModule  # noqa: F401,E402

DefaultActorCriticModule = RLModule
MultiAgentRLModule = MultiRLModule
SingleAgentRLModuleSpec = RLModuleSpec
MultiAgentRLModuleSpec = MultiRLModuleSpec
