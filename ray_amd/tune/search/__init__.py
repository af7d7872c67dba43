from ray_amd.tune.search.sample import (choice, grid_search, lograndint, loguniform,  # noqa
                                        qlograndint, qloguniform, qrandint, qrandn, quniform,
                                        randint, randn, sample_from, uniform)
from ray_amd.tune.tuner import (BasicVariantGenerator, ConcurrencyLimiter, Repeater,  # noqa
                                Searcher)
from ray_amd.tune.search.model_based import (BayesOptSearch, HyperOptSearch,  # noqa
                                             OptunaSearch, TPESearch)
