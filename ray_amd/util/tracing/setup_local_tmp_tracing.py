"""``ray.util.tracing.setup_local_tmp_tracing`` (reference path): the startup hook that
exports spans to ``/tmp/spans`` (``RAY_AMD_TRACING_DIR`` overrides)::

    ray_amd.init(_tracing_startup_hook=
                 "ray_amd.util.tracing.setup_local_tmp_tracing:setup_tracing")
"""

import os

from ray_amd.util.tracing import tracing_helper


def setup_tracing() -> None:
    tracing_helper.enable(os.environ.get("RAY_AMD_TRACING_DIR", "/tmp/spans"))
