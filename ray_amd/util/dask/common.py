"""Dask task-graph primitives, without dask itself (the classic graph spec).

A graph is a mapping key -> computation. A computation is a *task* — a tuple whose
first item is callable, the rest its arguments — a list of computations, a key of the
graph (an alias), or a literal. Keys are hashables (strings, or tuples such as
``("x", 0)``); a task's arguments reference other entries by key."""

from __future__ import annotations

from typing import Any, Dict, Hashable, Iterator


def istask(x) -> bool:
    return type(x) is tuple and len(x) > 0 and callable(x[0])


def _ishashable(x) -> bool:
    try:
        hash(x)
        return True
    except TypeError:
        return False


def iskey(x, dsk) -> bool:
    return _ishashable(x) and x in dsk


def deps_of(comp, dsk) -> Iterator[Hashable]:
    """Keys of ``dsk`` that computation ``comp`` reads (each once, in first-use order)."""
    seen = set()
    stack = [comp]
    out = []
    while stack:
        c = stack.pop()
        if istask(c):
            stack.extend(reversed(c[1:]))
        elif isinstance(c, list):
            stack.extend(reversed(c))
        elif iskey(c, dsk):
            if c not in seen:
                seen.add(c)
                out.append(c)
    return iter(out)


def evaluate(comp, values: Dict[Hashable, Any]):
    """The value of a computation given its dependencies' values (dask's _execute_task)."""
    if istask(comp):
        fn, args = comp[0], comp[1:]
        return fn(*(evaluate(a, values) for a in args))
    if isinstance(comp, list):
        return [evaluate(c, values) for c in comp]
    if _ishashable(comp) and comp in values:
        return values[comp]
    return comp


def toposort(dsk, targets) -> list:
    """The keys needed for ``targets``, dependencies first (iterative DFS; raises on a
    cycle)."""
    order, state = [], {}
    for t in targets:
        if state.get(t) == 2:
            continue
        stack = [(t, iter(deps_of(dsk[t], dsk)))]
        state[t] = 1
        while stack:
            k, it = stack[-1]
            nxt = next(it, None)
            if nxt is None:
                stack.pop()
                state[k] = 2
                order.append(k)
            elif state.get(nxt) == 1:
                raise RuntimeError(f"cycle in the task graph at key {nxt!r}")
            elif state.get(nxt) is None:
                state[nxt] = 1
                stack.append((nxt, iter(deps_of(dsk[nxt], dsk))))
    return order


def flatten_keys(keys):
    """The leaf keys of a (nested list) keys spec."""
    if isinstance(keys, list):
        for k in keys:
            yield from flatten_keys(k)
    else:
        yield keys


def pack(keys, values):
    """Rebuild the nested list structure of ``keys`` from a key -> value mapping."""
    if isinstance(keys, list):
        return [pack(k, values) for k in keys]
    return values[keys]
