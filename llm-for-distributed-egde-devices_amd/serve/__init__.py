"""Serving / communication layer: gRPC TimeService + REST (reference-compatible), gRPC tensor
stage transport for the CPU edge pipeline, and the request-serving engine."""
from .time_service import get_current_time, make_server, now_string  # noqa: F401
