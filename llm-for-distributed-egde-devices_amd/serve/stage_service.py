"""gRPC activation transport between pipeline stages (CPU / edge configuration).

BASELINE.json config 1: "GPT-2-small 2-stage layer split over localhost gRPC on CPU".  The
reference only *intends* to deploy models across Jetson / x86 nodes over gRPC/TCP
(review1.pptx s7-s9); its gRPC service carries a time string.  Here a stage server
hosts layers [first, last) (+ head), keeps per-request KV caches and speaks the ``edgellm.Stage``
protocol (serve/proto/edgellm_stage.proto, hand-encoded protobuf):

  client (stage 0: embedding + layers [0, k))  --StageForward(hidden)-->  server (layers [k, L) + head)
                                               <--StageReply(tokens)---

Robustness (absent in the reference): per-call deadlines, bounded exponential
retry, idempotent replay (a retried (seq_id, step) returns the cached reply instead of
re-applying the step) and a fault injector that drops / delays messages for tests.
On MI355X the same stage split runs over RCCL P2P (edgellm.parallel.pipeline).
"""
from __future__ import annotations

import random
import threading
import time
from concurrent import futures
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import grpc
import numpy as np
import torch

from .. import ops
from ..engine.generate import GenerationResult, SamplingParams
from ..engine.kv_cache import KVCache
from ..models.decoder import AttnCtx, DecoderLM
from . import wire

SERVICE = "edgellm.Stage"
METHOD = "Forward"
FULL_METHOD = f"/{SERVICE}/{METHOD}"
KIND_PREFILL, KIND_DECODE, KIND_RESET = 0, 1, 2

_DTYPES = {"bfloat16": torch.bfloat16, "float32": torch.float32, "float16": torch.float16, "int64": torch.int64,
           "int32": torch.int32}


# ----------------------------------------------------------------------------------- codec
def encode_tensor(t: torch.Tensor) -> bytes:
    t = t.detach().contiguous().cpu()
    name = str(t.dtype).replace("torch.", "")
    raw = t.view(torch.int16).numpy().tobytes() if t.dtype == torch.bfloat16 else t.numpy().tobytes()
    return wire.field_packed_varints(1, list(t.shape)) + wire.field_string(2, name) + wire.field_bytes(3, raw)


def decode_tensor(data: bytes) -> torch.Tensor:
    f = wire.decode(data)
    shape = wire.unpack_varints(f[1][0]) if 1 in f else []
    name = f[2][0].decode() if 2 in f else "float32"
    raw = f[3][0] if 3 in f else b""
    if name == "bfloat16":
        arr = np.frombuffer(raw, dtype=np.int16).copy()
        return torch.from_numpy(arr).view(torch.bfloat16).reshape(shape)
    np_dt = {"float32": np.float32, "float16": np.float16, "int64": np.int64, "int32": np.int32}[name]
    return torch.from_numpy(np.frombuffer(raw, dtype=np_dt).copy()).reshape(shape)


def _f32(x: float) -> bytes:
    return np.float32(x).tobytes()


def encode_sampling(sp: SamplingParams, seed: int) -> bytes:
    out = b""
    for num, v in ((1, sp.temperature), (3, sp.top_p), (4, sp.repetition_penalty)):
        if v:
            out += wire._varint(num << 3 | wire.I32) + _f32(v)
    out += wire.field_varint(2, sp.top_k or 0) + wire.field_varint(5, int(sp.do_sample)) + wire.field_varint(6, seed)
    return out


def decode_sampling(data: bytes):
    f = wire.decode(data)
    g = lambda n, d=0.0: float(np.frombuffer(int(f[n][0]).to_bytes(4, "little"), np.float32)[0]) if n in f else d  # noqa: E731
    sp = SamplingParams(max_new_tokens=0, temperature=g(1), top_k=int(f.get(2, [0])[0]), top_p=g(3, 1.0),
                        repetition_penalty=g(4, 1.0), do_sample=bool(f.get(5, [0])[0]))
    return sp, int(f.get(6, [0])[0])


@dataclass
class StageForward:
    seq_id: int
    step: int
    kind: int
    hidden: Optional[torch.Tensor] = None
    start_pos: int = 0
    sampling: Optional[SamplingParams] = None
    seed: int = 0
    prompt_ids: Optional[torch.Tensor] = None

    def encode(self) -> bytes:
        out = wire.field_varint(1, self.seq_id) + wire.field_varint(2, self.step) + wire.field_varint(3, self.kind)
        if self.hidden is not None:
            out += wire.field_bytes(4, encode_tensor(self.hidden))
        out += wire.field_varint(5, self.start_pos)
        if self.sampling is not None:
            out += wire.field_bytes(6, encode_sampling(self.sampling, self.seed))
        if self.prompt_ids is not None:
            out += wire.field_bytes(7, encode_tensor(self.prompt_ids))
        return out

    @classmethod
    def decode(cls, data: bytes) -> "StageForward":
        f = wire.decode(data)
        m = cls(seq_id=f.get(1, [0])[0], step=f.get(2, [0])[0], kind=f.get(3, [0])[0], start_pos=f.get(5, [0])[0])
        if 4 in f:
            m.hidden = decode_tensor(f[4][0])
        if 6 in f:
            m.sampling, m.seed = decode_sampling(f[6][0])
        if 7 in f:
            m.prompt_ids = decode_tensor(f[7][0])
        return m


def encode_reply(hidden: Optional[torch.Tensor] = None, tokens: Optional[Sequence[int]] = None,
                 error: str = "") -> bytes:
    out = b""
    if hidden is not None:
        out += wire.field_bytes(1, encode_tensor(hidden))
    if tokens is not None:
        out += wire.field_packed_varints(2, list(tokens))
    return out + wire.field_string(3, error)


def decode_reply(data: bytes):
    f = wire.decode(data)
    hidden = decode_tensor(f[1][0]) if 1 in f else None
    tokens = wire.unpack_varints(f[2][0]) if 2 in f else None
    err = f[3][0].decode() if 3 in f else ""
    return hidden, tokens, err


# ----------------------------------------------------------------------------------- faults
class FaultInjector:
    """Drops (raises UNAVAILABLE-like errors) or delays a fraction of messages — tests only."""

    def __init__(self, drop_prob: float = 0.0, delay_s: float = 0.0, delay_prob: float = 0.0, seed: int = 0,
                 drop_first_n: int = 0):
        self.drop_prob, self.delay_s, self.delay_prob = drop_prob, delay_s, delay_prob
        self.rng = random.Random(seed)
        self.drop_first_n = drop_first_n
        self.dropped = 0

    def before_send(self):
        if self.drop_first_n > 0:
            self.drop_first_n -= 1
            self.dropped += 1
            raise ConnectionError("injected drop")
        if self.drop_prob and self.rng.random() < self.drop_prob:
            self.dropped += 1
            raise ConnectionError("injected drop")
        if self.delay_prob and self.rng.random() < self.delay_prob:
            time.sleep(self.delay_s)


# ----------------------------------------------------------------------------------- server
class StageServer:
    """Hosts one pipeline stage behind gRPC.  Thread-safe (one forward at a time)."""

    def __init__(self, model: DecoderLM, max_seq: int = 1024, max_requests: int = 8, server_delay: float = 0.0):
        self.model = model
        self.max_seq = max_seq
        self.lock = threading.Lock()
        self.slots: Dict[int, dict] = {}
        self.max_requests = max_requests
        self.server_delay = server_delay
        self.rope = model.rope_table()
        self.calls = 0
        self.replays = 0

    def _slot(self, seq_id: int, batch: int) -> dict:
        s = self.slots.get(seq_id)
        if s is None or s["kv"].max_batch != batch:
            if len(self.slots) >= self.max_requests:
                self.slots.pop(next(iter(self.slots)))
            s = {"kv": KVCache(self.model.cfg, batch, self.max_seq, getattr(self.model, "kv_first", self.model.first), self.model.last,
                               self.model.dtype, self.model.device), "last": None}
            self.slots[seq_id] = s
        return s

    def forward(self, msg: StageForward) -> bytes:
        with self.lock:
            self.calls += 1
            if self.server_delay:
                time.sleep(self.server_delay)
            if msg.kind == KIND_RESET:
                self.slots.pop(msg.seq_id, None)
                return encode_reply()
            hidden = msg.hidden.to(self.model.device)
            B = msg.prompt_ids.shape[0] if msg.prompt_ids is not None else None
            slot = self.slots.get(msg.seq_id)
            if slot is not None and slot["last"] is not None and slot["last"][0] == (msg.step, msg.kind):
                self.replays += 1                  # retried message: replay, do not re-apply
                return slot["last"][1]
            if msg.kind == KIND_PREFILL:
                slot = self._slot(msg.seq_id, B)
                slot["B"] = B
                T = hidden.shape[0] // B
            else:
                slot = self.slots[msg.seq_id]
                B, T = slot["B"], 1
            sp = torch.full((B,), msg.start_pos, dtype=torch.int32, device=self.model.device)
            mode = "prefill" if msg.kind == KIND_PREFILL else "decode"
            ctx = AttnCtx(mode, B, T, sp, sp + T, msg.start_pos + T, slot["kv"], self.rope)
            out = self.model(None, ctx, hidden=hidden)
            if self.model.has_head:
                if msg.kind == KIND_PREFILL:
                    slot["seen"] = torch.zeros(B, self.model.cfg.vocab_size, dtype=torch.uint8, device=out.device)
                    slot["seen"].scatter_(1, msg.prompt_ids.to(out.device).long(), 1)
                    slot["sampling"] = msg.sampling
                    slot["rng"] = torch.tensor([msg.seed & 0x7FFFFFFF, 0], dtype=torch.int32, device=out.device)
                spp = slot["sampling"]
                slot["rng"][1] = msg.step
                tok = ops.sample(out, slot["seen"], spp.temperature, spp.top_k, spp.top_p,
                                 spp.repetition_penalty, slot["rng"], spp.do_sample)
                reply = encode_reply(tokens=tok.tolist())
            else:
                reply = encode_reply(hidden=out)
            slot["last"] = ((msg.step, msg.kind), reply)
            return reply

    def handler(self) -> grpc.GenericRpcHandler:
        def fn(request: bytes, context) -> bytes:
            try:
                return self.forward(StageForward.decode(request))
            except Exception as e:  # report to the caller instead of killing the worker
                return encode_reply(error=f"{type(e).__name__}: {e}")
        return grpc.method_handlers_generic_handler(SERVICE, {
            METHOD: grpc.unary_unary_rpc_method_handler(fn, request_deserializer=None, response_serializer=None)})


def serve_stage(stage: StageServer, port: int = 0, host: str = "127.0.0.1", max_workers: int = 4,
                with_time_service: bool = True) -> grpc.Server:
    from .time_service import time_service_handler
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers),
                         options=[("grpc.max_receive_message_length", 256 << 20),
                                  ("grpc.max_send_message_length", 256 << 20)])
    handlers = [stage.handler()] + ([time_service_handler()] if with_time_service else [])
    server.add_generic_rpc_handlers(handlers)
    server.port = server.add_insecure_port(f"{host}:{port}")
    server.start()
    return server


# ----------------------------------------------------------------------------------- client
class RemoteStage:
    def __init__(self, target: str, timeout: float = 30.0, retries: int = 3, backoff: float = 0.05,
                 faults: Optional[FaultInjector] = None):
        self.target, self.timeout, self.retries, self.backoff = target, timeout, retries, backoff
        self.faults = faults
        self.channel = grpc.insecure_channel(target, options=[("grpc.max_receive_message_length", 256 << 20),
                                                              ("grpc.max_send_message_length", 256 << 20)])
        self.call = self.channel.unary_unary(FULL_METHOD, request_serializer=None, response_deserializer=None)
        self.retried = 0

    def forward(self, msg: StageForward):
        data = msg.encode()
        last = None
        for attempt in range(self.retries + 1):
            try:
                if self.faults is not None:
                    self.faults.before_send()
                hidden, tokens, err = decode_reply(self.call(data, timeout=self.timeout))
                if err:
                    raise RuntimeError(f"remote stage error: {err}")
                return hidden, tokens
            except (grpc.RpcError, ConnectionError) as e:
                last = e
                self.retried += 1
                time.sleep(self.backoff * (2 ** attempt))
        raise RuntimeError(f"stage {self.target} failed after {self.retries + 1} attempts") from last

    def close(self):
        self.channel.close()


class EdgePipeline:
    """Local first stage + remote stages over gRPC; batch generation with the same sampling
    semantics as the single-device engine."""

    def __init__(self, first: DecoderLM, remotes: List[RemoteStage], max_seq: int = 1024):
        assert first.has_embed and not first.has_head
        self.first, self.remotes, self.max_seq = first, remotes, max_seq
        self.rope = first.rope_table()
        self._seq = random.Random().randrange(1 << 40)

    @torch.no_grad()
    def generate(self, prompts: Sequence[Sequence[int]], sampling: SamplingParams, seed: int = 0) -> GenerationResult:
        plens = {len(p) for p in prompts}
        assert len(plens) == 1, "EdgePipeline batches equal-length prompts"
        B, T = len(prompts), plens.pop()
        self._seq += 1
        seq_id = self._seq
        kv = KVCache(self.first.cfg, B, self.max_seq, getattr(self.first, "kv_first", self.first.first), self.first.last, self.first.dtype,
                     self.first.device)
        ids = torch.tensor(prompts, dtype=torch.long, device=self.first.device)
        t0 = time.perf_counter()
        out_tokens: List[List[int]] = [[] for _ in range(B)]
        step_ms: List[float] = []
        pos, cur, t_prefill = 0, ids, 0.0
        for step in range(sampling.max_new_tokens):
            ts = time.perf_counter()
            Tn = cur.shape[1]
            sp = torch.full((B,), pos, dtype=torch.int32, device=self.first.device)
            mode = "prefill" if step == 0 else "decode"
            ctx = AttnCtx(mode, B, Tn, sp, sp + Tn, pos + Tn, kv, self.rope)
            h = self.first(cur, ctx)
            kind = KIND_PREFILL if step == 0 else KIND_DECODE
            msg = StageForward(seq_id, step, kind, h, pos, sampling if step == 0 else None, seed,
                               ids.cpu() if step == 0 else None)
            toks = None
            for r in self.remotes:
                hid, toks = r.forward(msg)
                if hid is not None:
                    msg = StageForward(seq_id, step, kind, hid, pos, msg.sampling, seed, msg.prompt_ids)
            assert toks is not None, "the last remote stage must own the LM head"
            for b, t in enumerate(toks):
                out_tokens[b].append(int(t))
            pos += Tn
            cur = torch.tensor(toks, dtype=torch.long, device=self.first.device).view(B, 1)
            dt = time.perf_counter() - ts
            if step == 0:
                t_prefill = dt
            else:
                step_ms.append(dt * 1e3)
        for r in self.remotes:
            try:
                r.forward(StageForward(seq_id, 0, KIND_RESET))
            except RuntimeError:
                pass
        el = time.perf_counter() - t0
        return GenerationResult(out_tokens, [T] * B, el, t_prefill, el - t_prefill, step_ms)
