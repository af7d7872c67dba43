"""Distributed tracing (reference: python/ray/util/tracing/). See ``tracing_helper``."""

from ray_amd.util.tracing.tracing_helper import (disable, enable, is_enabled,  # noqa: F401
                                                 read_spans, span)
