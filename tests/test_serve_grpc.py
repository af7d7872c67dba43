"""Serve gRPC ingress (modelled on python/ray/serve/tests/test_grpc.py). protoc is not
in the image, so the servicer function below is written the way protoc's *_pb2_grpc
output is (add_<Service>Servicer_to_server registering generic method handlers) with
plain-bytes serialisers instead of protobuf messages."""

import json
import socket

import grpc
import pytest

import ray_amd as ray
from ray_amd import serve


def add_EchoServicer_to_server(servicer, server):
    handlers = {
        "Upper": grpc.unary_unary_rpc_method_handler(
            servicer.Upper, request_deserializer=lambda b: b.decode(),
            response_serializer=lambda s: s.encode()),
        "Count": grpc.unary_stream_rpc_method_handler(
            servicer.Count, request_deserializer=lambda b: int(b.decode()),
            response_serializer=lambda s: str(s).encode()),
    }
    server.add_generic_rpc_handlers(
        (grpc.method_handlers_generic_handler("test.EchoService", handlers),))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def grpc_port():
    ray.init(num_cpus=6)
    port = _free_port()
    serve.start(http_options={"port": _free_port()},
                grpc_options=serve.gRPCOptions(
                    port=port, grpc_servicer_functions=[add_EchoServicer_to_server]))
    yield port
    serve.shutdown()
    ray.shutdown()


@serve.deployment
class Echo:
    def __init__(self, suffix):
        self.suffix = suffix

    def Upper(self, req):
        return req.upper() + self.suffix

    def Count(self, n):
        return list(range(n))


def test_grpc_unary_stream_and_routing(grpc_port):
    serve.run(Echo.bind("!"), name="app1", route_prefix="/a1")
    serve.run(Echo.bind("?"), name="app2", route_prefix="/a2")
    ch = grpc.insecure_channel(f"127.0.0.1:{grpc_port}")
    upper = ch.unary_unary("/test.EchoService/Upper", request_serializer=str.encode,
                           response_deserializer=bytes.decode)
    assert upper("hi", metadata=(("application", "app1"),), timeout=30) == "HI!"
    assert upper("hi", metadata=(("application", "app2"),), timeout=30) == "HI?"
    with pytest.raises(grpc.RpcError) as ei:
        upper("hi", timeout=30)  # two apps and no application metadata
    assert ei.value.code() == grpc.StatusCode.NOT_FOUND
    count = ch.unary_stream("/test.EchoService/Count", request_serializer=lambda n: str(n).encode(),
                            response_deserializer=lambda b: int(b.decode()))
    assert list(count(4, metadata=(("application", "app1"),), timeout=30)) == [0, 1, 2, 3]
    ident = (lambda b: b)
    health = ch.unary_unary("/ray.serve.RayServeAPIService/Healthz",
                            request_serializer=ident, response_deserializer=ident)
    assert health(b"", timeout=30) == b"success"
    apps = ch.unary_unary("/ray.serve.RayServeAPIService/ListApplications",
                          request_serializer=ident, response_deserializer=ident)
    assert json.loads(apps(b"", timeout=30)) == ["app1", "app2"]
