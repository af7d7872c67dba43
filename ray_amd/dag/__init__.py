"""Lazy task/actor DAGs (reference: python/ray/dag/{dag_node,function_node,class_node,
input_node,output_node}.py).

``f.bind(x)`` builds a node; ``node.execute(*inputs)`` submits the graph with
each node's upstream results passed as ObjectRefs (so data never returns to the
driver between stages)."""

from __future__ import annotations

import uuid


class DAGNode:
    def __init__(self, args, kwargs, options):
        self._bound_args = tuple(args)
        self._bound_kwargs = dict(kwargs)
        self._bound_options = dict(options or {})
        self._stable_uuid = uuid.uuid4().hex

    def get_args(self):
        return self._bound_args

    def get_kwargs(self):
        return self._bound_kwargs

    def get_options(self):
        return self._bound_options

    def _children(self):
        out = []
        for a in list(self._bound_args) + list(self._bound_kwargs.values()):
            if isinstance(a, DAGNode):
                out.append(a)
            elif isinstance(a, (list, tuple)):
                out.extend(x for x in a if isinstance(x, DAGNode))
            elif isinstance(a, dict):
                out.extend(x for x in a.values() if isinstance(x, DAGNode))
        return out

    def _resolve(self, v, cache, inputs):
        if isinstance(v, DAGNode):
            return v._exec(cache, inputs)
        if isinstance(v, list):
            return [self._resolve(x, cache, inputs) for x in v]
        if isinstance(v, tuple):
            return tuple(self._resolve(x, cache, inputs) for x in v)
        if isinstance(v, dict):
            return {k: self._resolve(x, cache, inputs) for k, x in v.items()}
        return v

    def _exec(self, cache, inputs):
        key = self._stable_uuid
        if key not in cache:
            args = [self._resolve(a, cache, inputs) for a in self._bound_args]
            kwargs = {k: self._resolve(v, cache, inputs) for k, v in self._bound_kwargs.items()}
            cache[key] = self._execute_impl(args, kwargs, cache, inputs)
        return cache[key]

    def execute(self, *args, **kwargs):
        cache = {}
        out = self._exec(cache, (args, kwargs))
        self._last_cache = cache
        return out

    # ------------------------------------------------ reference DAGNode helpers
    def get_stable_uuid(self) -> str:
        return self._stable_uuid

    def get_other_args_to_resolve(self) -> dict:
        return dict(getattr(self, "_bound_other_args_to_resolve", {}) or {})

    def get_object_refs_from_last_execute(self) -> dict:
        """{node uuid: the value (ObjectRef for remote nodes) the last ``execute`` got}."""
        return dict(getattr(self, "_last_cache", {}) or {})

    def clear_cache(self) -> None:
        self._last_cache = {}

    def apply_recursive(self, fn):
        """Post-order: ``fn`` on every upstream node then on this one; returns ``fn(self)``
        of a copy whose children were replaced by their ``fn`` results."""
        memo = {}

        def visit(node):
            key = node._stable_uuid
            if key in memo:
                return memo[key]

            def sub(v):
                if isinstance(v, DAGNode):
                    return visit(v)
                if isinstance(v, list):
                    return [sub(x) for x in v]
                if isinstance(v, tuple):
                    return tuple(sub(x) for x in v)
                if isinstance(v, dict):
                    return {k: sub(x) for k, x in v.items()}
                return v

            import copy

            clone = copy.copy(node)
            clone._bound_args = tuple(sub(a) for a in node._bound_args)
            clone._bound_kwargs = {k: sub(v) for k, v in node._bound_kwargs.items()}
            memo[key] = fn(clone)
            return memo[key]

        return visit(self)

    def apply_functional(self, source_input_list, predictate_fn, apply_fn):
        """``apply_fn(x)`` for every ``x`` in ``source_input_list`` (recursing into lists
        / tuples / dicts) for which ``predictate_fn(x)``; returns the transformed copy."""
        def go(v):
            if predictate_fn(v):
                return apply_fn(v)
            if isinstance(v, list):
                return [go(x) for x in v]
            if isinstance(v, tuple):
                return tuple(go(x) for x in v)
            if isinstance(v, dict):
                return {k: go(x) for k, x in v.items()}
            return v

        return go(source_input_list)

    def _execute_impl(self, args, kwargs, cache, inputs):
        raise NotImplementedError

    def experimental_compile(self, *, enable_asyncio: bool = False,
                             _submit_timeout=None, _buffer_size_bytes=None,
                             _max_inflight_executions=None, _get_timeout=None, **kw):
        """Compile into channel-connected persistent actor loops (reference:
        dag_node.py:experimental_compile). See ``compiled_dag_node``."""
        from .compiled_dag_node import CompiledDAG

        return CompiledDAG(self, buffer_size_bytes=_buffer_size_bytes,
                           max_inflight_executions=_max_inflight_executions,
                           submit_timeout=_submit_timeout, get_timeout=_get_timeout,
                           enable_asyncio=enable_asyncio)

    def with_tensor_transport(self, transport: str = "auto", **kw):
        """Move torch tensors in this node's output through the HBM object store
        (device-to-device, zero-copy readers) instead of host memory."""
        self._tensor_transport = transport
        return self

    with_type_hint = with_tensor_transport


class InputNode(DAGNode):
    def __init__(self, *a, **k):
        super().__init__((), {}, {})

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def __getitem__(self, key):
        return InputAttributeNode(self, key)

    def __getattr__(self, key):
        if key.startswith("_"):
            raise AttributeError(key)
        return InputAttributeNode(self, key, attr=True)

    def _execute_impl(self, args, kwargs, cache, inputs):
        a, k = inputs
        if len(a) == 1 and not k:
            return a[0]
        if not a and k:
            return k
        return a


class InputAttributeNode(DAGNode):
    def __init__(self, parent, key, attr=False):
        super().__init__((), {}, {})
        self._parent = parent
        self._key = key
        self._attr = attr

    def _execute_impl(self, args, kwargs, cache, inputs):
        a, k = inputs
        if isinstance(self._key, int):
            return a[self._key]
        if self._key in k:
            return k[self._key]
        v = self._parent._exec(cache, inputs)
        return getattr(v, self._key) if self._attr else v[self._key]


class FunctionNode(DAGNode):
    def __init__(self, fn, args, kwargs, options):
        super().__init__(args, kwargs, options)
        self._fn = fn

    def _execute_impl(self, args, kwargs, cache, inputs):
        return self._fn._remote(args, kwargs, self._bound_options)


class ClassNode(DAGNode):
    def __init__(self, cls, args, kwargs, options):
        super().__init__(args, kwargs, options)
        self._cls = cls

    def _execute_impl(self, args, kwargs, cache, inputs):
        return self._cls._remote(args, kwargs, self._bound_options)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return _UnboundClassMethod(self, name)


class _UnboundClassMethod:
    def __init__(self, cls_node, name):
        self._cls_node = cls_node
        self._name = name

    def bind(self, *args, **kwargs):
        return ClassMethodNode(self._cls_node, self._name, args, kwargs, {})

    def options(self, **opts):
        parent = self

        class _O:
            def bind(self, *a, **k):
                return ClassMethodNode(parent._cls_node, parent._name, a, k, opts)

        return _O()


class ClassMethodNode(DAGNode):
    def __init__(self, actor_or_node, method, args, kwargs, options):
        super().__init__(args, kwargs, options)
        self._actor = actor_or_node
        self._method = method

    def _children(self):
        c = super()._children()
        if isinstance(self._actor, DAGNode):
            c.append(self._actor)
        return c

    def _execute_impl(self, args, kwargs, cache, inputs):
        handle = self._actor._exec(cache, inputs) if isinstance(self._actor, DAGNode) \
            else self._actor
        return getattr(handle, self._method).options(**self._bound_options).remote(*args,
                                                                                  **kwargs)


class MultiOutputNode(DAGNode):
    def __init__(self, outputs):
        super().__init__((list(outputs),), {}, {})

    def _execute_impl(self, args, kwargs, cache, inputs):
        return list(args[0])


DAGNODE_TYPE_KEY = "__dag_node_type__"
PARENT_CLASS_NODE_KEY = "__parent_class_node__"
PREV_CLASS_METHOD_CALL_KEY = "__prev_class_method_call__"


class DAGInputData:
    """The positional + keyword input of one DAG execution (what an InputNode resolves to;
    reference: dag/input_node.py DAGInputData)."""

    def __init__(self, *args, **kwargs):
        self._args = list(args)
        self._kwargs = kwargs

    def __getitem__(self, key):
        return self._args[key] if isinstance(key, int) else self._kwargs[key]

    def __getattr__(self, key):
        try:
            return self.__dict__["_kwargs"][key]
        except KeyError:
            raise AttributeError(key) from None


def _label(n: DAGNode) -> str:
    if isinstance(n, InputNode):
        return "InputNode"
    if isinstance(n, InputAttributeNode):
        return f"Input[{getattr(n, '_key', '?')!r}]"
    if isinstance(n, MultiOutputNode):
        return "MultiOutputNode"
    for attr in ("_body", "_func", "_method_name", "_cls"):
        v = getattr(n, attr, None)
        if v is not None:
            return f"{type(n).__name__}({getattr(v, '__name__', v)})"
    return type(n).__name__


def to_dot(dag: DAGNode) -> str:
    """Graphviz DOT text of a DAG (nodes by stable uuid, edges child -> parent)."""
    seen, lines = {}, ["digraph dag {", "  rankdir=LR;"]
    stack = [dag]
    while stack:
        n = stack.pop()
        if n._stable_uuid in seen:
            continue
        seen[n._stable_uuid] = n
        lines.append(f'  "{n._stable_uuid}" [label="{_label(n)}"];')
        for c in n._children():
            lines.append(f'  "{c._stable_uuid}" -> "{n._stable_uuid}";')
            stack.append(c)
    lines.append("}")
    return "\n".join(lines)


def plot(dag: DAGNode, to_file: str | None = None):
    """Write the DAG as Graphviz DOT (``.dot``/``.gv``), or render it (``.png``/``.svg``/
    ``.pdf``) through the ``dot`` binary when installed; returns the DOT text."""
    import os
    import shutil
    import subprocess

    text = to_dot(dag)
    if to_file is None:
        return text
    ext = os.path.splitext(to_file)[1].lstrip(".").lower()
    if ext in ("dot", "gv", ""):
        with open(to_file, "w") as f:
            f.write(text)
        return text
    exe = shutil.which("dot")
    if exe is None:
        raise ImportError(f"rendering .{ext} needs the graphviz 'dot' binary; write a .dot file "
                          "instead")
    subprocess.run([exe, f"-T{ext}", "-o", to_file], input=text.encode(), check=True)
    return text


def __getattr__(name):
    if name in ("CompiledDAG", "CompiledDAGRef", "CompiledDAGFuture"):
        from . import compiled_dag_node

        return getattr(compiled_dag_node, name)
    raise AttributeError(name)


__all__ = ["DAGNode", "InputNode", "FunctionNode", "ClassNode", "ClassMethodNode",
           "MultiOutputNode", "InputAttributeNode", "CompiledDAG",
           "CompiledDAGRef", "CompiledDAGFuture", "DAGInputData", "plot", "DAGNODE_TYPE_KEY",
           "PARENT_CLASS_NODE_KEY", "PREV_CLASS_METHOD_CALL_KEY"]
