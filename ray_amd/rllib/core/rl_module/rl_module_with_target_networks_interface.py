"""``RLModuleWithTargetNetworksInterface`` (reference path): modules with target networks
(DQN / SAC-style) implement ``get_target_network_pairs`` and
``forward_target``; ray_amd's QModule / TwinQ keep their targets in the learner."""

import abc


class RLModuleWithTargetNetworksInterface(abc.ABC):
    @abc.abstractmethod
    def get_target_network_pairs(self):
        """[(main_net, target_net), ...] to sync / Polyak-average."""

    @abc.abstractmethod
    def forward_target(self, batch, **kwargs):
        """The forward pass through the target network(s)."""

    def make_target_networks(self) -> None:
        """Create the target copies (called once after setup)."""
