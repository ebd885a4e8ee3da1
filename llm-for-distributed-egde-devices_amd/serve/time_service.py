"""gRPC TimeService + REST time endpoint, compatible with the reference's comm demo.

Reference: ``TimeService.GetCurrentTime(TimeRequest) -> TimeResponse{string current_time}``
served on ``[::]:50051`` by a 10-worker thread pool (Code/gRPC/server.py:9-19, proto :5-13),
client ``client.py:7-11`` (hard-wired to 192.168.1.101:50051), REST ``GET /`` ->
``{"current_time": "%Y-%m-%d %H:%M:%S"}`` on 0.0.0.0:8000 (rest_api.py:9-15).

Same service/method/message names and field numbers (wire-compatible with protoc stubs built
from the reference .proto), plus what the reference lacks: a configurable target
(no hard-coded IP), client deadlines and bounded retries.
"""
from __future__ import annotations

import time
from concurrent import futures
from typing import Optional

import grpc

from . import wire

SERVICE = "TimeService"
METHOD = "GetCurrentTime"
FULL_METHOD = f"/{SERVICE}/{METHOD}"
TIME_FORMAT = "%Y-%m-%d %H:%M:%S"


def now_string() -> str:
    return time.strftime(TIME_FORMAT)


def encode_time_response(current_time: str) -> bytes:
    return wire.field_string(1, current_time)


def decode_time_response(data: bytes) -> str:
    f = wire.decode(data)
    return f.get(1, [b""])[0].decode("utf-8")


def _get_current_time(request: bytes, context) -> bytes:  # TimeRequest{} has no fields
    return encode_time_response(now_string())


def time_service_handler() -> grpc.GenericRpcHandler:
    return grpc.method_handlers_generic_handler(SERVICE, {
        METHOD: grpc.unary_unary_rpc_method_handler(_get_current_time, request_deserializer=None,
                                                    response_serializer=None)})


def make_server(port: int = 50051, host: str = "[::]", max_workers: int = 10, extra_handlers=()) -> grpc.Server:
    """Thread-pool server (server.py:14-16).  Returns the started server; ``server.port`` holds
    the bound port (pass port=0 for an ephemeral one)."""
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers))
    server.add_generic_rpc_handlers((time_service_handler(), *extra_handlers))
    bound = server.add_insecure_port(f"{host}:{port}")
    server.start()
    server.port = bound
    return server


def get_current_time(target: str = "127.0.0.1:50051", timeout: float = 5.0, retries: int = 3,
                     backoff: float = 0.2) -> str:
    """Unary call with a deadline and bounded exponential-backoff retry."""
    last: Optional[Exception] = None
    for attempt in range(retries + 1):
        try:
            with grpc.insecure_channel(target) as ch:
                call = ch.unary_unary(FULL_METHOD, request_serializer=None, response_deserializer=None)
                return decode_time_response(call(b"", timeout=timeout))
        except grpc.RpcError as e:  # UNAVAILABLE / DEADLINE_EXCEEDED
            last = e
            time.sleep(backoff * (2 ** attempt))
    raise RuntimeError(f"TimeService at {target} unreachable after {retries + 1} attempts") from last


def serve(port: int = 50051, host: str = "[::]") -> None:  # pragma: no cover - CLI
    server = make_server(port, host)
    print(f"gRPC Server running on port {server.port}...")
    server.wait_for_termination()
