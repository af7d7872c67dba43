"""``train_one_step`` (reference: rllib/execution/train_ops.py): one learner update of an
algorithm on a sampled batch, then a weight sync to the env runners."""

from __future__ import annotations


def train_one_step(algorithm, train_batch, policies_to_train=None) -> dict:
    lg = algorithm.learner_group
    res = lg.update_from_batch(train_batch)
    algorithm._sync_weights(algorithm.get_weights())
    return res
