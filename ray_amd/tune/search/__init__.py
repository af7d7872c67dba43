from ray_amd.tune.search.sample import (choice, grid_search, lograndint, loguniform,  # noqa
                                        qlograndint, qloguniform, qrandint, qrandn, quniform,
                                        randint, randn, sample_from, uniform)
from ray_amd.tune.tuner import (BasicVariantGenerator, ConcurrencyLimiter, Repeater,  # noqa
                                Searcher)
from ray_amd.tune.search.model_based import (BayesOptSearch, HyperOptSearch,  # noqa
                                             OptunaSearch, TPESearch)

UNRESOLVED_SEARCH_SPACE = ("You passed a `{par}` parameter to {cls} that contained unresolved "
                           "search space definitions. {cls} should however be instantiated "
                           "with fully configured search spaces only.")
UNDEFINED_SEARCH_SPACE = ("Trying to sample a configuration from {cls}, but no search space has "
                          "been defined.")
UNDEFINED_METRIC_MODE = ("Trying to sample a configuration from {cls}, but the `metric` "
                         "({metric}) or `mode` ({mode}) parameters have not been set.")


class SearchAlgorithm:
    """Legacy interface above Searcher: produces trials (``next_trial``) and hears results."""

    def set_search_properties(self, metric, mode, config, **spec):
        return True

    def add_configurations(self, experiments):
        raise NotImplementedError

    def next_trial(self):
        raise NotImplementedError

    def on_trial_result(self, trial_id, result):
        pass

    def on_trial_complete(self, trial_id, result=None, error=False):
        pass

    def is_finished(self) -> bool:
        raise NotImplementedError

    def set_finished(self):
        self._finished = True


class SearchGenerator(SearchAlgorithm):
    """Adapts a ``Searcher`` to the SearchAlgorithm interface (Tuner accepts either)."""

    def __init__(self, searcher: Searcher):
        self.searcher = searcher
        self._finished = False
        self._count = 0

    def set_search_properties(self, metric, mode, config, **spec):
        return self.searcher.set_search_properties(metric, mode, config)

    def next_trial(self):
        cfg = self.searcher.suggest(f"trial_{self._count:05d}")
        if cfg is None:
            self._finished = True
            return None
        self._count += 1
        return cfg

    def suggest(self, trial_id):
        return self.searcher.suggest(trial_id)

    def on_trial_result(self, trial_id, result):
        if hasattr(self.searcher, "on_trial_result"):
            self.searcher.on_trial_result(trial_id, result)

    def on_trial_complete(self, trial_id, result=None, error=False):
        self.searcher.on_trial_complete(trial_id, result=result, error=error)

    def is_finished(self) -> bool:
        return self._finished

    def __getattr__(self, name):
        return getattr(self.searcher, name)


# name -> searcher (reference: tune/search/__init__.py SEARCH_ALG_IMPORT / create_searcher)
def _searcher_registry():
    from ray_amd.tune.search import model_based as mb

    reg = {"variant_generator": BasicVariantGenerator, "random": BasicVariantGenerator}
    for name, attr in (("bayesopt", "BayesOptSearch"), ("hyperopt", "HyperOptSearch"),
                       ("optuna", "OptunaSearch"), ("tpe", "TPESearch")):
        cls = globals().get(attr) or getattr(mb, attr, None)
        if cls is not None:
            reg[name] = cls
    return reg


def create_searcher(search_alg, **kwargs):
    """A searcher by name ("variant_generator", "random", "bayesopt", "hyperopt",
    "optuna", "tpe"), constructed with ``kwargs``; a Searcher instance passes through."""
    if not isinstance(search_alg, str):
        return search_alg
    reg = _searcher_registry()
    key = search_alg.lower()
    if key not in reg:
        raise ValueError(f"Search algorithm must be one of {sorted(reg)}. Got: {search_alg}")
    return reg[key](**kwargs)
