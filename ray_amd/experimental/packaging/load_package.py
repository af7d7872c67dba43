"""Ray code packages (reference: python/ray/experimental/packaging/load_package.py).

A package is a directory with a YAML config::

    name: my_pkg
    description: what it does
    interface_file: interface.py        # defines @ray.remote functions / actor classes
    runtime_env: {pip: [...], env_vars: {...}}

``load_package(path)`` imports the interface file and hands back its remote functions and
actor classes bound to the package's runtime env (``working_dir`` defaults to the
package directory, so the workers import the same code). GitHub URLs are refused: this
framework has no network fetch of code."""

from __future__ import annotations

import importlib.util
import os

import yaml


class _RuntimePackage:
    def __init__(self, name: str, desc: str, interface_file: str, runtime_env: dict):
        from ray_amd.actor import ActorClass
        from ray_amd.remote_function import RemoteFunction

        self._name = name
        self._description = desc
        self._interface_file = interface_file
        self._runtime_env = runtime_env
        if not os.path.exists(interface_file):
            raise ValueError(f"interface file does not exist: {interface_file}")
        spec = importlib.util.spec_from_file_location(name, interface_file)
        module = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(module)
        self._module = module
        for sym in dir(module):
            if sym.startswith("_"):
                continue
            v = getattr(module, sym)
            if isinstance(v, (RemoteFunction, ActorClass)):
                v = v.options(runtime_env=runtime_env)
            setattr(self, sym, v)

    def __repr__(self):
        return f"ray_amd.experimental.packaging.Package(name={self._name!r})"


def load_package(config_path: str) -> _RuntimePackage:
    """Load the package described by ``config_path`` (a local YAML file)."""
    if str(config_path).startswith("http"):
        raise ValueError("load_package() takes a local package config (no network fetch)")
    config_path = os.path.expanduser(config_path)
    if not os.path.exists(config_path):
        raise ValueError(f"Config file does not exist: {config_path}")
    with open(config_path) as f:
        config = yaml.safe_load(f)
    base = os.path.abspath(os.path.dirname(config_path))
    renv = dict(config.get("runtime_env") or {})
    renv.setdefault("working_dir", base)
    conda = os.path.join(base, "conda.yaml")
    if os.path.exists(conda):
        if "conda" in renv:
            raise ValueError("Both conda.yaml and conda: section found in package")
        with open(conda) as f:
            renv["conda"] = yaml.safe_load(f)
    return _RuntimePackage(config["name"], config.get("description", ""),
                           os.path.join(base, config["interface_file"]), renv)
