"""Minimal protobuf (proto3) wire codec — enough for the services here, no protoc needed.

``grpc_tools``/``protoc`` are not available in this environment, so the
messages are encoded by hand; the encodings are byte-compatible with protoc output for the
same .proto definitions (see ``serve/proto/*.proto``), so stock gRPC clients interoperate.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

VARINT, I64, LEN, I32 = 0, 1, 2, 5


def _varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = result = 0
    while True:
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7


def field_varint(num: int, v: int) -> bytes:
    return _varint(num << 3 | VARINT) + _varint(v) if v else b""


def field_bytes(num: int, data: bytes) -> bytes:
    return _varint(num << 3 | LEN) + _varint(len(data)) + data if data else b""


def field_string(num: int, s: str) -> bytes:
    return field_bytes(num, s.encode("utf-8"))


def field_packed_varints(num: int, vals: List[int]) -> bytes:
    if not vals:
        return b""
    return field_bytes(num, b"".join(_varint(v) for v in vals))


def decode(buf: bytes) -> Dict[int, list]:
    """field number -> list of raw values (ints for varint/fixed, bytes for length-delimited)."""
    out: Dict[int, list] = {}
    i = 0
    n = len(buf)
    while i < n:
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == VARINT:
            v, i = _read_varint(buf, i)
        elif wt == LEN:
            ln, i = _read_varint(buf, i)
            v = bytes(buf[i:i + ln])
            i += ln
        elif wt == I64:
            v = int.from_bytes(buf[i:i + 8], "little")
            i += 8
        elif wt == I32:
            v = int.from_bytes(buf[i:i + 4], "little")
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        out.setdefault(num, []).append(v)
    return out


def unpack_varints(data: bytes) -> List[int]:
    vals, i = [], 0
    while i < len(data):
        v, i = _read_varint(data, i)
        if v >= 1 << 63:
            v -= 1 << 64
        vals.append(v)
    return vals
