"""Batched generation engine: prefill + HIP-graph-captured decode loop.

Replaces HF ``model.generate`` as called by the reference (``get_response`` /
``refine_summary``, combine_model_fp_updated.py:86-135).  Differences by design:
  * KV cache preallocated, head-major (no per-step ``torch.cat``);
  * one decode step = one HIP graph replay: embedding -> layers -> head -> fused sampler ->
    position/step counters, all on device; no host sync per token (EOS is polled every
    ``eos_check_every`` steps from a device token buffer);
  * seedable, counter-based sampling (reference sets no seed anywhere — SURVEY §2.2).
Timing follows both reference TPS definitions (``GenerationResult``).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch

from .. import ops
from ..utils.tracing import debug_sync, trace_range
from ..models.decoder import AttnCtx, DecoderLM
from .kv_cache import KVCache

GRAPH_BUCKET = 256


@dataclass
class SamplingParams:
    max_new_tokens: int = 200
    temperature: float = 0.7
    top_k: int = 50
    top_p: float = 0.9
    repetition_penalty: float = 1.1
    do_sample: bool = True

    @classmethod
    def from_config(cls, s) -> "SamplingParams":
        return cls(s.max_new_tokens, s.temperature, s.top_k, s.top_p, s.repetition_penalty,
                   getattr(s, "do_sample", True))

    def key(self):
        return (self.temperature, self.top_k, self.top_p, self.repetition_penalty, self.do_sample)


@dataclass
class GenerationResult:
    tokens: List[List[int]]          # generated ids per sequence (EOS included if produced)
    prompt_lens: List[int]
    elapsed_s: float                 # prefill + decode wall time (reference timer span)
    prefill_s: float
    decode_s: float
    step_ms: List[float] = field(default_factory=list)  # per decode-step latency (device events)

    @property
    def num_generated(self) -> int:
        return sum(len(t) for t in self.tokens)

    def tps_generated(self) -> float:
        """Generated tokens / time (combiners, combine_model_fp_updated.py:106-108)."""
        return self.num_generated / self.elapsed_s if self.elapsed_s > 0 else 0.0

    def tps_incl_prompt(self) -> float:
        """(prompt + generated) tokens / time (single-model scripts, Llama_bf16_updated.py:89-90)."""
        n = self.num_generated + sum(self.prompt_lens)
        return n / self.elapsed_s if self.elapsed_s > 0 else 0.0

    def p50_ms(self) -> float:
        if not self.step_ms:
            return float("nan")
        s = sorted(self.step_ms)
        return s[len(s) // 2]


def needs_host_sampler(sp: SamplingParams, V: int) -> bool:
    """True when the fused sampler cannot express the config (top-p without top-k, or
    top-k > 1024): the step then syncs with the host and cannot be graph-captured."""
    if not sp.do_sample or sp.temperature <= 0:
        return False
    full = (sp.top_k is None or sp.top_k <= 0 or sp.top_k >= V)
    if full and (sp.top_p is None or sp.top_p >= 1.0):
        return False
    return not (sp.top_k and 0 < sp.top_k <= 1024 and sp.top_k < V)


class _DecodeState:
    """Static device buffers read and advanced by the (captured) decode step."""

    def __init__(self, B: int, V: int, max_new: int, device):
        self.tok = torch.zeros(B, dtype=torch.long, device=device)
        self.pos = torch.zeros(B, dtype=torch.int32, device=device)       # position of tok
        self.seq_lens = torch.ones(B, dtype=torch.int32, device=device)   # pos + 1
        self.rng = torch.zeros(2, dtype=torch.int32, device=device)       # [seed, step]
        self.step = torch.zeros(1, dtype=torch.long, device=device)       # column in out
        self.out = torch.zeros(B, max_new, dtype=torch.long, device=device)
        self.seen = torch.zeros(B, V, dtype=torch.uint8, device=device)
        self.ctr = torch.zeros(1, dtype=torch.int32, device=device)       # sampler arrival counter


class Generator:
    def __init__(self, model: DecoderLM, max_batch: int = 1, max_seq: Optional[int] = None,
                 use_graphs: Optional[bool] = None, eos_check_every: int = 8, kv: Optional[KVCache] = None,
                 prefill_chunk: Optional[int] = None, kv_dtype: str = "bf16"):
        """``kv_dtype``: "bf16" or "int8" (per-(token, head) scaled int8 KV cache, engine.kv_cache)."""
        assert model.has_embed and model.has_head, "Generator needs a full model (use parallel.pipeline for stages)"
        self.model = model
        self.cfg = model.cfg
        self.device = model.device
        max_seq = min(max_seq or self.cfg.max_position_embeddings, self.cfg.max_position_embeddings)
        self.max_seq = max_seq
        if kv is None:
            # a model split over several devices (parallel.split.SplitLM) brings per-stage caches
            kv = (model.make_kv(max_batch, max_seq, kv_dtype) if hasattr(model, "make_kv") else
                  KVCache(self.cfg, max_batch, max_seq, device=self.device, dtype=model.dtype, kv_dtype=kv_dtype))
        self.kv = kv
        self.rope = model.rope_table(self.device)
        # HeadInfer (edgellm.offload) caches carry an attention hook and a prefill chunk size
        self.attn_hook = getattr(self.kv, "attn_hook", None)
        self.prefill_chunk = prefill_chunk or (getattr(self.kv, "chunk_size", None) if self.attn_hook is not None
                                               else None)
        self.use_graphs = (self.device.type == "cuda") if use_graphs is None else use_graphs
        self.eos_check_every = eos_check_every
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self._pool = None
        self._warm = False                # a decode step of the current state ran eagerly
        self._state: Optional[_DecodeState] = None
        # batch-1 decode through the persistent one-launch engine (engine/b1_engine.py): needs every CU
        # of the GPU, so generators that decode concurrently on one device (co_generate, LaneGenerator)
        # turn it off
        from . import b1_engine
        self.b1 = self.device.type == "cuda" and b1_engine.enabled()

    # ------------------------------------------------------------------ forward pieces
    @torch.no_grad()
    def prefill(self, ids: torch.Tensor, row0: int = 0, start: int = 0,
                lens: Optional[Sequence[int]] = None) -> torch.Tensor:
        """ids [B, T] into cache rows [row0, row0+B) at positions start.. ; returns the logits of
        each row's last real token [B, V].  ``lens``: ragged prompts right-padded to T (one pass
        for the whole batch; AttnCtx.last_pos)."""
        B, T = ids.shape
        assert start + T <= self.max_seq, "prompt exceeds the KV cache"
        if self.prefill_chunk and T > self.prefill_chunk:     # chunked prefill (HeadInfer)
            assert lens is None or len(set(lens)) == 1, "chunked prefill takes equal-length prompts"
            out = None
            for c0 in range(0, T, self.prefill_chunk):
                out = self.prefill(ids[:, c0:c0 + self.prefill_chunk], row0, start + c0)
            return out
        sp = torch.full((B,), start, dtype=torch.int32, device=self.device)
        last = None
        if lens is not None and len(set(lens)) > 1:
            last = torch.tensor([n - 1 for n in lens], dtype=torch.long, device=self.device)
        ctx = AttnCtx("prefill", B, T, sp, sp + T, start + T, self.kv.rows(row0, row0 + B), self.rope,
                      attn_hook=self.attn_hook, last_pos=last)
        with trace_range(f"prefill.B{B}.T{T}"):
            out = self.model(ids, ctx)
        debug_sync("prefill")
        return out

    def _decode_step(self, st: _DecodeState, B: int, max_len: int, sp: SamplingParams):
        ctx = AttnCtx("decode", B, 1, st.pos, st.seq_lens, max_len, self.kv.rows(0, B), self.rope,
                      attn_hook=self.attn_hook, b1=self.b1 and B == 1)
        logits = self.model(st.tok.view(B, 1), ctx)
        ops.sample_advance(logits, st.seen, sp.temperature, sp.top_k, sp.top_p, sp.repetition_penalty, st.rng,
                           st.tok, st.out, st.step, st.pos, st.seq_lens, st.ctr, sp.do_sample)

    def _graph_for(self, st: _DecodeState, B: int, bucket: int, sp: SamplingParams):
        key = (B, bucket, sp.key(), id(st))
        g = self._graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, pool=self._pool):
                self._decode_step(st, B, bucket, sp)
            if self._pool is None:
                self._pool = g.pool()
            self._graphs[key] = g
        return g

    def reset_graphs(self):
        self._graphs.clear()
        self._pool = None
        self._warm = False

    # ------------------------------------------------------------------ generate
    @torch.no_grad()
    def start(self, prompts: Sequence[Sequence[int]], sampling: SamplingParams, seed: int = 0) -> None:
        """Prefill ``prompts`` and sample their first token; decode then advances with ``step``."""
        B = len(prompts)
        assert B <= self.kv.max_batch
        V = self.cfg.vocab_size
        plens = [len(p) for p in prompts]
        max_new = sampling.max_new_tokens
        assert max(plens) + max_new <= self.max_seq, "prompt + max_new_tokens exceeds max_seq"
        assert self.attn_hook is None or len(set(plens)) == 1, "HeadInfer offload batches equal-length prompts"
        st = self._state
        if st is None or st.tok.shape[0] != B or st.out.shape[1] < max_new:
            self.reset_graphs()
            st = self._state = _DecodeState(B, V, max_new, self.device)
        st.seen.zero_()
        st.out.zero_()
        st.step.zero_()
        st.rng[0] = seed & 0x7FFFFFFF
        st.rng[1] = 0
        cuda = self.device.type == "cuda"
        if cuda:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        # one batched pass; ragged prompts are right-padded to the longest (AttnCtx.last_pos), except
        # under HeadInfer's chunked prefill, which takes one pass per sequence (own cache row)
        if len(set(plens)) == 1:
            logits = self.prefill(torch.tensor(prompts, dtype=torch.long, device=self.device), 0, 0)
        elif not self.prefill_chunk:
            T = max(plens)
            pad = [list(p) + [0] * (T - len(p)) for p in prompts]
            logits = self.prefill(torch.tensor(pad, dtype=torch.long, device=self.device), 0, 0, lens=plens)
        else:
            logits = torch.cat([self.prefill(torch.tensor([p], dtype=torch.long, device=self.device), b, 0)
                                for b, p in enumerate(prompts)], 0)
        for b, p in enumerate(prompts):
            st.seen[b, torch.tensor(p, dtype=torch.long, device=self.device)] = 1
        st.pos.copy_(torch.tensor(plens, dtype=torch.int32, device=self.device))
        st.seq_lens.copy_(st.pos + 1)
        nxt = ops.sample(logits, st.seen, sampling.temperature, sampling.top_k, sampling.top_p,
                         sampling.repetition_penalty, st.rng, sampling.do_sample)
        st.tok.copy_(nxt)
        st.out[:, 0] = nxt
        st.rng[1] = 1
        st.step.fill_(1)
        if cuda:
            torch.cuda.synchronize()
        self._run = dict(B=B, plens=plens, sampling=sampling, t0=t0, t_prefill=time.perf_counter() - t0,
                         prefill_logits=logits, produced=1, host_max=max(plens), events=[], cuda=cuda,
                         graphs_ok=self.use_graphs and cuda and self.graph_safe_for(B)
                         and not needs_host_sampler(sampling, V))

    @property
    def graph_safe(self) -> bool:
        return getattr(self.kv, "graph_safe", True) and \
            all(getattr(m, "graph_safe", True) for m in self.model.modules())

    def graph_safe_for(self, B: int) -> bool:
        """graph_safe, counting modules that are capturable up to a batch size (``graph_safe_rows``)."""
        return getattr(self.kv, "graph_safe", True) and \
            all(getattr(m, "graph_safe", True) or getattr(m, "graph_safe_rows", 0) >= B for m in self.model.modules())

    @torch.no_grad()
    def step(self, n: int = 1, record_latency: bool = True) -> int:
        """Advance every sequence by up to ``n`` decode tokens; returns tokens produced so far."""
        r, st = self._run, self._state
        B, sampling = r["B"], r["sampling"]
        for _ in range(n):
            if r["produced"] >= sampling.max_new_tokens:
                break
            max_len = r["host_max"] + 1
            with trace_range(f"decode.B{B}"):
                if r["graphs_ok"]:
                    bucket = min(self.max_seq, ((max_len + GRAPH_BUCKET - 1) // GRAPH_BUCKET) * GRAPH_BUCKET)
                    if not self._warm:
                        # first step of this decode state runs eagerly (lazy weight packs, workspace
                        # allocations, autotune choices happen outside any capture); every later
                        # step replays the captured graph of its length bucket
                        self._decode_step(st, B, bucket, sampling)
                        self._warm = True
                    else:
                        self._graph_for(st, B, bucket, sampling).replay()
                else:
                    self._decode_step(st, B, max_len, sampling)
            debug_sync("decode step")
            if record_latency and r["cuda"]:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                r["events"].append(ev)
            r["produced"] += 1
            r["host_max"] += 1
        return r["produced"]

    @torch.no_grad()
    def precapture(self, n_steps: int) -> int:
        """Capture the decode graphs of every length bucket the next ``n_steps`` will touch
        (capture records, it does not execute), so no capture lands in a timed region."""
        r = self._run
        if not r["graphs_ok"] or not self._warm:
            return 0
        lo = r["host_max"] + 1
        hi = min(self.max_seq, lo + n_steps)
        made = 0
        b = ((lo + GRAPH_BUCKET - 1) // GRAPH_BUCKET) * GRAPH_BUCKET
        while True:
            bucket = min(self.max_seq, b)
            key = (r["B"], bucket, r["sampling"].key(), id(self._state))
            if key not in self._graphs:
                self._graph_for(self._state, r["B"], bucket, r["sampling"])
                made += 1
            if b >= hi:
                break
            b += GRAPH_BUCKET
        return made

    def all_hit(self, eos_token_id: int) -> bool:
        st, r = self._state, self._run
        return bool((st.out[:, :r["produced"]] == eos_token_id).any(1).all().item())

    @torch.no_grad()
    def collect(self, eos_token_id: Optional[int] = None, stop_at_eos: bool = True) -> GenerationResult:
        r, st = self._run, self._state
        if r["cuda"]:
            torch.cuda.synchronize()
        t_end = time.perf_counter()
        for eng in getattr(self.model, "_b1_engines", {}).values():
            eng.check()
        toks = []
        for row in st.out[:, :r["produced"]].tolist():
            if stop_at_eos and eos_token_id is not None and eos_token_id in row:
                row = row[:row.index(eos_token_id) + 1]
            toks.append(row)
        ev = r["events"]
        step_ms = [ev[i - 1].elapsed_time(ev[i]) for i in range(1, len(ev))] if ev else []
        return GenerationResult(toks, r["plens"], t_end - r["t0"], r["t_prefill"], t_end - r["t0"] - r["t_prefill"],
                                step_ms)

    @torch.no_grad()
    def generate(self, prompts: Sequence[Sequence[int]], sampling: SamplingParams, seed: int = 0,
                 eos_token_id: Optional[int] = None, stop_at_eos: bool = True,
                 record_step_latency: bool = True) -> GenerationResult:
        self.start(prompts, sampling, seed)
        while self._run["produced"] < sampling.max_new_tokens:
            self.step(self.eos_check_every, record_step_latency)
            if stop_at_eos and eos_token_id is not None and self.all_hit(eos_token_id):
                break
        return self.collect(eos_token_id, stop_at_eos)


class LaneGenerator:
    """``lanes`` independent Generators on one GPU (own KV rows, decode state, graphs and graph
    memory pools) whose decode steps are replayed on ``lanes`` HIP streams, so one lane's
    latency-bound kernels (norms, attention tails, kernel boundaries) overlap another lane's
    weight streaming.  Each step advances every lane by one token.  Prompts are dealt to the
    lanes in contiguous chunks; lane i samples with seed + 7919 * i."""

    def __init__(self, model: DecoderLM, lanes: int = 2, max_batch: int = 1, max_seq: Optional[int] = None,
                 use_graphs: Optional[bool] = None, **kw):
        assert lanes >= 1
        self.lanes = [Generator(model, max_batch=max_batch, max_seq=max_seq, use_graphs=use_graphs, **kw)
                      for _ in range(lanes)]
        for g in self.lanes:
            g.b1 = False                   # concurrent lanes: the one-launch engine needs every CU
        self.cuda = model.device.type == "cuda"
        self.streams = [torch.cuda.Stream(model.device) for _ in range(lanes)] if self.cuda else [None] * lanes

    def _on(self, i):
        return torch.cuda.stream(self.streams[i]) if self.cuda else _null_ctx()

    @torch.no_grad()
    def start(self, prompts: Sequence[Sequence[int]], sampling: SamplingParams, seed: int = 0) -> None:
        L = len(self.lanes)
        per = (len(prompts) + L - 1) // L
        for i, g in enumerate(self.lanes):
            chunk = list(prompts[i * per:(i + 1) * per])
            assert chunk, "fewer prompts than lanes"
            g.start(chunk, sampling, seed + 7919 * i)
        self._t_prefill = sum(g._run["t_prefill"] for g in self.lanes)

    def precapture(self, n_steps: int) -> int:
        return sum(g.precapture(n_steps) for g in self.lanes)

    @torch.no_grad()
    def step(self, n: int = 1, record_latency: bool = True) -> None:
        if self.cuda:
            cur = torch.cuda.current_stream()
            for s in self.streams:
                s.wait_stream(cur)
        for _ in range(n):
            for i, g in enumerate(self.lanes):
                with self._on(i):
                    g.step(1, record_latency)
        if self.cuda:
            for s in self.streams:
                cur.wait_stream(s)

    def step_latencies_ms(self) -> List[float]:
        """Per-lane intervals between consecutive recorded steps (device events)."""
        out: List[float] = []
        for g in self.lanes:
            ev = g._run["events"]
            out += [ev[i - 1].elapsed_time(ev[i]) for i in range(1, len(ev))]
        return out

    def collect(self, eos_token_id: Optional[int] = None, stop_at_eos: bool = True) -> List[GenerationResult]:
        return [g.collect(eos_token_id, stop_at_eos) for g in self.lanes]


@torch.no_grad()
def co_generate(jobs: Sequence[tuple], eos_check_every: int = 8) -> List[GenerationResult]:
    """Run several Generators that share one GPU CONCURRENTLY: ``jobs`` = [(generator, prompts,
    sampling, seed, eos_token_id)].  Every generator gets its own HIP stream; the prefills run
    one after another, each generator's decode graphs are captured up front (single host thread,
    so no capture overlaps another stream's launches), then one host loop issues ``eos_check_every``
    graph replays per generator round-robin — while the host waits on one generator's EOS flag the
    others' queued steps keep the GPU busy, and their weight streams overlap each other's latency-
    bound kernels.  This is how ensemble agents placed on the same device decode side by side
    (orchestrator.ensemble) instead of one after another."""
    if not jobs:
        return []
    gens = [j[0] for j in jobs]
    if len(gens) > 1:
        for g in gens:
            g.b1 = False                   # concurrent decode: the one-launch engine needs every CU
    cuda = gens[0].device.type == "cuda"
    streams = [torch.cuda.Stream(g.device) for g in gens] if cuda else [None] * len(gens)
    on = (lambda i: torch.cuda.stream(streams[i])) if cuda else (lambda i: _null_ctx())
    for g, prompts, sp, seed, _ in jobs:
        g.start(prompts, sp, seed)
    if cuda:
        cur = torch.cuda.current_stream()
        for st in streams:
            st.wait_stream(cur)
    for i, (g, _, sp, _, _) in enumerate(jobs):
        with on(i):
            g.step(2)                      # eager warm-up step + first capture, then every bucket
            g.precapture(sp.max_new_tokens)
    active = list(range(len(jobs)))
    while active:
        for i in list(active):
            g, _, sp, _, eos = jobs[i]
            with on(i):
                g.step(eos_check_every)
                done = g._run["produced"] >= sp.max_new_tokens or (eos is not None and g.all_hit(eos))
            if done:
                active.remove(i)
    if cuda:
        for st in streams:
            cur.wait_stream(st)
    return [g.collect(j[4]) for g, j in zip(gens, jobs)]


class _null_ctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
