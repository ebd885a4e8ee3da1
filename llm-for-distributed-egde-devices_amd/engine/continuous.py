"""Iteration-level (continuous) batching over the cache rows of one Generator.

``Generator.generate`` runs a batch to completion: a request that arrives one step after a batch
started waits for the whole batch, and a short answer holds its row until the longest one ends.
``SlotDecoder`` instead treats the B cache rows as slots: a request is prefilled into a free slot
and its first token sampled while the other slots are mid-decode, every decode step advances all
occupied slots by one token (one graph replay for the whole batch, ragged lengths through the
per-row ``seq_lens``), and a slot is released the moment its request hits EOS or its
``max_new_tokens`` — so the next queued request starts on the next step.

Device state per slot: ``pos`` / ``seq_lens`` advance by the ``active`` mask inside the captured
step (a free slot stays at position 0 with one key, so it never writes past its row), ``seen``
(repetition penalty) and the row of ``out`` are reset on admission.  Generated tokens land in a
session-wide ``out[B, width]`` at the step column; slot r's tokens are the columns from its
admission on.  One sampling configuration per session (the fused sampler takes one per launch):
``ServingEngine`` opens a new session when the queue head needs another one.  The sampling noise
is keyed by (seed, row, step) of the session, so a sampled request's tokens depend on its slot
and admission step (greedy requests are exactly those of a solo run).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch

from .. import ops
from ..models.decoder import AttnCtx
from ..utils.tracing import trace_range
from .generate import GRAPH_BUCKET, GenerationResult, Generator, SamplingParams, _DecodeState, needs_host_sampler


@dataclass
class _Slot:
    tag: object
    prompt_len: int
    max_new: int
    eos: Optional[int]
    col0: int                      # out column of the first token
    produced: int = 1
    t0: float = 0.0
    t_first: float = 0.0
    tokens: List[int] = field(default_factory=list)


class SlotDecoder:
    def __init__(self, gen: Generator, sampling: SamplingParams, seed: int = 0, width: int = 2048,
                 max_batch: Optional[int] = None):
        assert gen.attn_hook is None, "continuous batching needs per-row cache lengths (no HeadInfer offload)"
        self.gen, self.sp = gen, sampling
        self.model, self.cfg, self.device = gen.model, gen.cfg, gen.device
        # slots = the operator's batch cap (ServingEngine max_batch), at most the cache rows
        self.B = min(int(max_batch), gen.kv.max_batch) if max_batch else gen.kv.max_batch
        self.V = self.cfg.vocab_size
        self.width = width
        self.st = _DecodeState(self.B, self.V, width, self.device)
        self.active = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self.st.rng[0] = seed & 0x7FFFFFFF
        self.st.rng[1] = 1
        self.st.step.fill_(1)
        self.col = 1                                   # host mirror of st.step
        self.slots: List[Optional[_Slot]] = [None] * self.B
        self.host_len = [1] * self.B                   # keys each row attends over next step
        self.cuda = self.device.type == "cuda"
        self.use_graphs = gen.use_graphs and self.cuda and gen.graph_safe_for(self.B) and \
            not needs_host_sampler(sampling, self.V)
        self._graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self._pool = None
        self._warm = False
        self.steps = 0

    # ------------------------------------------------------------------ slots
    def free_slots(self) -> List[int]:
        return [r for r, s in enumerate(self.slots) if s is None]

    def busy(self) -> bool:
        return any(s is not None for s in self.slots)

    def can_admit(self, prompt_len: int, max_new: int) -> bool:
        return bool(self.free_slots()) and prompt_len + max_new <= self.gen.max_seq and \
            self.col - 1 + max_new < self.width

    @torch.no_grad()
    def admit(self, ids: Sequence[int], max_new: int, eos: Optional[int] = None, tag=None) -> int:
        """Prefill ``ids`` into a free slot and sample its first token; returns the slot."""
        assert self.can_admit(len(ids), max_new), "no slot / cache room for this request"
        r = self.free_slots()[0]
        st, sp = self.st, self.sp
        t0 = time.perf_counter()
        x = torch.tensor([list(ids)], dtype=torch.long, device=self.device)
        with trace_range("serve.admit"):
            logits = self.gen.prefill(x, r, 0)
            st.seen[r].zero_()
            st.seen[r, x[0]] = 1
            nxt = ops.sample(logits, st.seen[r:r + 1], sp.temperature, sp.top_k, sp.top_p, sp.repetition_penalty,
                             st.rng, sp.do_sample)
        st.tok[r:r + 1].copy_(nxt)
        st.out[r].zero_()
        st.out[r, self.col - 1:self.col].copy_(nxt)
        st.pos[r] = len(ids)
        st.seq_lens[r] = len(ids) + 1
        self.active[r] = 1
        self.host_len[r] = len(ids) + 1
        self.slots[r] = _Slot(tag, len(ids), max_new, eos, self.col - 1, 1, t0, time.perf_counter())
        return r

    # ------------------------------------------------------------------ decode
    def _decode_body(self, max_len: int):
        st, sp, B = self.st, self.sp, self.B
        ctx = AttnCtx("decode", B, 1, st.pos, st.seq_lens, max_len, self.gen.kv.rows(0, B), self.gen.rope)
        logits = self.model(st.tok.view(B, 1), ctx)
        nxt = ops.sample(logits, st.seen, sp.temperature, sp.top_k, sp.top_p, sp.repetition_penalty, st.rng,
                         sp.do_sample)
        # free slots stay at position 0 (increments = the active flags)
        ops.decode_advance(nxt, st.tok, st.out, st.step, st.pos, st.seq_lens, st.rng, self.active)

    def _bucket(self, n: int) -> int:
        return min(self.gen.max_seq, ((n + GRAPH_BUCKET - 1) // GRAPH_BUCKET) * GRAPH_BUCKET)

    @torch.no_grad()
    def step(self, n: int = 1) -> int:
        """``n`` decode steps of every occupied slot (stops early once a slot reaches its token
        budget, so a finished request never decodes past it); returns the steps taken."""
        done = 0
        for _ in range(n):
            live = [r for r, s in enumerate(self.slots) if s is not None and s.produced < s.max_new]
            if not live or self.col >= self.width:
                break
            max_len = max(self.host_len)
            with trace_range(f"serve.decode.B{self.B}"):
                if not self.use_graphs:
                    self._decode_body(max_len)
                elif not self._warm:
                    self._warm = True
                    self._decode_body(self._bucket(max_len))
                else:
                    b = self._bucket(max_len)
                    g = self._graphs.get(b)
                    if g is None:
                        g = torch.cuda.CUDAGraph()
                        torch.cuda.synchronize()
                        with torch.cuda.graph(g, pool=self._pool):
                            self._decode_body(b)
                        if self._pool is None:
                            self._pool = g.pool()
                        self._graphs[b] = g
                    g.replay()
            self.col += 1
            self.steps += 1
            done += 1
            for r, s in enumerate(self.slots):
                # a slot already at its budget rode along in the batched step (its row advanced on
                # device) but produced no token of its request: it is released by the next poll
                if s is not None and s.produced < s.max_new:
                    s.produced += 1
                if s is not None:
                    self.host_len[r] += 1
            if any(s is not None and s.produced >= s.max_new for s in self.slots):
                break
        return done

    @torch.no_grad()
    def poll(self) -> List[tuple]:
        """Release finished slots: [(tag, GenerationResult)] for requests that hit EOS or their
        token budget (one device -> host read of the occupied rows)."""
        occ = [r for r, s in enumerate(self.slots) if s is not None]
        if not occ:
            return []
        c0 = min(self.slots[r].col0 for r in occ)
        rows = self.st.out[occ, c0:self.col].tolist()
        now = time.perf_counter()
        out = []
        for r, row in zip(occ, rows):
            s = self.slots[r]
            toks = row[s.col0 - c0:s.col0 - c0 + min(s.produced, s.max_new)]
            hit = s.eos is not None and s.eos in toks
            if hit:
                toks = toks[:toks.index(s.eos) + 1]
            if hit or s.produced >= s.max_new:
                res = GenerationResult([toks], [s.prompt_len], now - s.t0, s.t_first - s.t0, now - s.t_first, [])
                out.append((s.tag, res))
                self.slots[r] = None
                self.active[r] = 0
                self.st.pos[r] = 0
                self.st.seq_lens[r] = 1
                self.host_len[r] = 1
        return out
