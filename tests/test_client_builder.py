"""ray.client() builder, RuntimeEnv validation, serve.HTTPOptions (reference:
python/ray/tests/test_client_builder.py, test_runtime_env.py)."""

import os

import pytest

import ray_amd as ray


def test_client_builder_runtime_env_http_options():
    from ray_amd.runtime_env import RuntimeEnv, RuntimeEnvConfig
    from ray_amd.serve import HTTPOptions

    env = RuntimeEnv(env_vars={"FOO": "bar"}, config={"setup_timeout_seconds": 10})
    assert env["env_vars"] == {"FOO": "bar"} and isinstance(env["config"], RuntimeEnvConfig)
    assert RuntimeEnv.deserialize(env.serialize())["env_vars"] == {"FOO": "bar"}
    with pytest.raises(ValueError):
        RuntimeEnv(pip=["x"], conda="y")
    with pytest.raises(TypeError):
        RuntimeEnv(env_vars={"A": 1})
    assert HTTPOptions(port=9000).to_dict()["port"] == 9000
    with pytest.raises(ValueError):
        HTTPOptions(location="Nowhere")
    with ray.client().namespace("ns1").env(env)._init_args(num_cpus=2).connect() as ctx:
        assert ray.is_initialized() and ctx.ray_version == ray.__version__

        @ray.remote
        def f():
            return os.environ.get("FOO")

        assert ray.get(f.remote()) == "bar"
        assert ray.get_runtime_context().namespace == "ns1"
    assert not ray.is_initialized()
