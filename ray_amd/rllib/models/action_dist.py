"""Old-stack action distributions (reference: python/ray/rllib/models/action_dist.py and
models/torch/torch_action_dist.py): built from a model's output ``inputs``; sample,
deterministic_sample, logp, entropy, kl, sampled_action_logp."""

from __future__ import annotations

import numpy as np
import torch


class ActionDistribution:
    def __init__(self, inputs, model=None):
        self.inputs = inputs
        self.model = model

    def sample(self):
        raise NotImplementedError

    def deterministic_sample(self):
        raise NotImplementedError

    def sampled_action_logp(self):
        raise NotImplementedError

    def logp(self, x):
        raise NotImplementedError

    def kl(self, other):
        raise NotImplementedError

    def entropy(self):
        raise NotImplementedError

    def multi_kl(self, other):
        return self.kl(other)

    def multi_entropy(self):
        return self.entropy()

    @staticmethod
    def required_model_output_shape(action_space, model_config):
        raise NotImplementedError


class TorchDistributionWrapper(ActionDistribution):
    def __init__(self, inputs, model=None):
        if not isinstance(inputs, torch.Tensor):
            inputs = torch.as_tensor(np.asarray(inputs), dtype=torch.float32)
        super().__init__(inputs, model)
        self.last_sample = None

    def logp(self, actions):
        return self.dist.log_prob(actions)

    def entropy(self):
        return self.dist.entropy()

    def kl(self, other):
        return torch.distributions.kl.kl_divergence(self.dist, other.dist)

    def sample(self):
        self.last_sample = self.dist.sample()
        return self.last_sample

    def sampled_action_logp(self):
        assert self.last_sample is not None, "sample() first"
        return self.logp(self.last_sample)


class TorchCategorical(TorchDistributionWrapper):
    def __init__(self, inputs, model=None, temperature: float = 1.0):
        super().__init__(inputs, model)
        self.dist = torch.distributions.Categorical(logits=self.inputs / temperature)

    def deterministic_sample(self):
        self.last_sample = self.dist.probs.argmax(dim=-1)
        return self.last_sample

    @staticmethod
    def required_model_output_shape(action_space, model_config=None):
        return int(action_space.n)


class TorchDiagGaussian(TorchDistributionWrapper):
    """Inputs: ``[mean, log_std]`` halves."""

    def __init__(self, inputs, model=None, *, action_space=None):
        super().__init__(inputs, model)
        mean, log_std = torch.chunk(self.inputs, 2, dim=-1)
        self.mean, self.log_std = mean, log_std
        self.dist = torch.distributions.Normal(mean, torch.exp(log_std))

    def deterministic_sample(self):
        self.last_sample = self.mean
        return self.last_sample

    def logp(self, actions):
        return self.dist.log_prob(actions).sum(-1)

    def entropy(self):
        return self.dist.entropy().sum(-1)

    def kl(self, other):
        return torch.distributions.kl.kl_divergence(self.dist, other.dist).sum(-1)

    @staticmethod
    def required_model_output_shape(action_space, model_config=None):
        return 2 * int(np.prod(action_space.shape))


class TorchDeterministic(TorchDistributionWrapper):
    def __init__(self, inputs, model=None):
        super().__init__(inputs, model)

    def deterministic_sample(self):
        return self.inputs

    def sample(self):
        self.last_sample = self.inputs
        return self.inputs

    def logp(self, x):
        return torch.zeros(self.inputs.shape[:-1], device=self.inputs.device)

    def sampled_action_logp(self):
        return self.logp(self.inputs)

    def entropy(self):
        return torch.zeros(self.inputs.shape[:-1], device=self.inputs.device)

    @staticmethod
    def required_model_output_shape(action_space, model_config=None):
        return int(np.prod(action_space.shape))
