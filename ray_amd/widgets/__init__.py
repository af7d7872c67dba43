"""Notebook display helpers (reference: python/ray/widgets/): HTML table reprs with a
plain-text fallback outside notebooks."""

from ray_amd.widgets.util import (Template, in_ipython_shell, in_notebook,  # noqa: F401
                                  make_table_html_repr, repr_with_fallback)
