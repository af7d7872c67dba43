"""HTML rendering for notebook reprs (reference: python/ray/widgets/{render,util}.py)."""

from __future__ import annotations

import html
from typing import Any, Optional


class Template:
    """A string template with ``{{ key }}`` placeholders (HTML-escaped on render unless
    the value is marked safe by wrapping it in ``Template.Safe``)."""

    class Safe(str):
        pass

    def __init__(self, text: str):
        self.text = text

    def render(self, **kwargs) -> str:
        out = self.text
        for k, v in kwargs.items():
            s = v if isinstance(v, Template.Safe) else html.escape(str(v))
            out = out.replace("{{ " + k + " }}", s).replace("{{" + k + "}}", s)
        return out


def make_table_html_repr(obj: Any, title: Optional[str] = None,
                         max_height: str = "none") -> str:
    """An HTML table of ``obj``'s public attributes (or a dict's items)."""
    items = obj.items() if isinstance(obj, dict) else \
        ((k, v) for k, v in vars(obj).items() if not k.startswith("_"))
    rows = "".join(f"<tr><td>{html.escape(str(k))}</td><td>{html.escape(str(v))}</td></tr>"
                   for k, v in items)
    head = f"<h3>{html.escape(title)}</h3>" if title else ""
    return (f'<div style="max-height:{max_height};overflow:auto">{head}'
            f"<table>{rows}</table></div>")


def _get_ipython_shell_name() -> str:
    try:
        from IPython import get_ipython

        sh = get_ipython()
        return type(sh).__name__ if sh is not None else ""
    except ImportError:
        return ""


def in_notebook(shell_name: Optional[str] = None) -> bool:
    return (shell_name if shell_name is not None else _get_ipython_shell_name()) == \
        "ZMQInteractiveShell"


def in_ipython_shell(shell_name: Optional[str] = None) -> bool:
    return (shell_name if shell_name is not None else _get_ipython_shell_name()) == \
        "TerminalInteractiveShell"


def repr_with_fallback(*notebook_deps):
    """Decorator for ``_repr_html_`` methods: outside a notebook it returns None so the
    plain ``__repr__`` is used."""

    def wrap(fn):
        def inner(self, *a, **k):
            if not in_notebook():
                return None
            return fn(self, *a, **k)

        inner.__name__ = fn.__name__
        inner.__doc__ = fn.__doc__
        return inner

    return wrap
