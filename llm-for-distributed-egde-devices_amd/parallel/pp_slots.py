"""Continuous (iteration-level) batching over the RCCL pipeline.

``PipelineGenerator.generate`` runs a static batch to completion on every stage: a request that
arrives while a long one decodes waits for it, and a short answer holds its rows until the
longest one ends.  The reference's server hands requests to a 10-thread pool and answers each
on its own (Code/gRPC/server.py:14); here the pipeline's ``M x b`` KV rows become SLOTS, as
``engine.continuous.SlotDecoder`` does on one GPU:

* ``PipelineSlotDecoder`` (driver, rank 0) has SlotDecoder's interface (``can_admit`` /
  ``admit`` / ``step`` / ``poll`` / ``busy``), so ``serve.server.ServingEngine`` drives either.
  Every call is one command broadcast to all ranks (``serve_workers`` runs it on theirs).
* ``admit``: the prompt is prefilled into one free row on every stage (hidden states hop stage
  to stage), the last stage samples the first token, and the row becomes ACTIVE.
* ``step(n)``: n decode rounds of ALL rows through the usual micro-batched tick schedule (rank
  r computes item i = k M + m at tick i + r; hidden states go r -> r + 1, the tokens sampled on
  the last stage come back to stage 0 one exchange later, M >= P keeps that ring full).  Free rows
  ride along at position 0 with one key; ``pos`` / ``seq_lens`` advance by the active flags
  (``ops.decode_advance``), so a free row never writes past its first cache slot.
* a request that hits EOS or its token budget is released by ``poll`` at the next command
  boundary; its row is admitted to the next queued request at once, while the other rows keep
  decoding.

One sampling configuration per session, as SlotDecoder (the fused sampler takes one per launch).
Decode steps run eagerly (no graph capture: the active set changes between commands).  Greedy
requests give exactly the tokens of a single-process ``Generator`` run.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from .. import ops
from ..engine.generate import GenerationResult, SamplingParams
from ..models.decoder import AttnCtx

CMD_SLOT_OPEN, CMD_SLOT_ADMIT, CMD_SLOT_STEP = 4, 5, 6
_HDR = 12


class _SlotSession:
    """The slots of one session on a member rank (stage state lives in ``eng.stage``)."""

    def __init__(self, eng, sampling: SamplingParams, seed: int, width: int):
        st = eng.stage
        self.eng, self.st, self.sp = eng, st, sampling
        self.M, self.b = st.M, st.b
        self.width = width
        dev = st.device
        self.active = [torch.zeros(self.b, dtype=torch.int32, device=dev) for _ in range(self.M)]
        self.host_active = [0] * (self.M * self.b)
        self.host_len = [1] * (self.M * self.b)        # keys each row attends over next (upper bound)
        self.col = 1                                   # out column the next decode round writes
        for m in range(self.M):
            st.pos[m].zero_()
            st.lens[m].fill_(1)
            st.tok[m].zero_()
        if st.is_last:
            V = st.cfg.vocab_size
            self.seen = [torch.zeros(self.b, V, dtype=torch.uint8, device=dev) for _ in range(self.M)]
            self.rng = [torch.tensor([(seed + 7919 * m) & 0x7FFFFFFF, 1], dtype=torch.int32, device=dev)
                        for m in range(self.M)]
            self.rng_adm = torch.tensor([(seed + 104729) & 0x7FFFFFFF, 0], dtype=torch.int32, device=dev)
            self.step_ = [torch.ones(1, dtype=torch.long, device=dev) for _ in range(self.M)]
            self.out = [torch.zeros(self.b, width, dtype=torch.long, device=dev) for _ in range(self.M)]

    # ------------------------------------------------------------------ admission
    @torch.no_grad()
    def admit(self, row: int, ids: torch.Tensor) -> torch.Tensor:
        """Prefill ``ids`` [T] into ``row`` on this stage; the last stage samples the first token.
        Returns a [1] token tensor (meaningful on the last stage)."""
        st, eng = self.st, self.eng
        m, i = divmod(row, self.b)
        T = int(ids.numel())
        dev = st.device
        H = st.cfg.hidden_size
        sp0 = torch.zeros(1, dtype=torch.int32, device=dev)
        ctx = AttnCtx("prefill", 1, T, sp0, sp0 + T, T, st.kv.rows(row, row + 1), st.rope)
        x_ids = ids.to(dev).view(1, T)
        hidden = None
        if not st.is_first:
            hidden = torch.empty(T, H, dtype=st.model.dtype, device=dev)
            st._exchange([], [(hidden, st.prev)])
        out = st.model(x_ids if st.is_first else None, ctx, hidden=hidden, logits="last")
        tok = torch.zeros(1, dtype=torch.long, device=eng.cdev)
        if not st.is_last:
            st._exchange([(out.contiguous(), st.next)], [])
        else:
            seen = self.seen[m][i:i + 1]
            seen.zero_()
            seen[0, x_ids[0]] = 1
            sp = self.sp
            nxt = ops.sample(out, seen, sp.temperature, sp.top_k, sp.top_p, sp.repetition_penalty, self.rng_adm,
                             sp.do_sample)
            self.rng_adm[1:].add_(1)
            st.tok[m][i:i + 1].copy_(nxt)
            self.out[m][i].zero_()
            self.out[m][i, self.col - 1] = nxt[0]
            tok.copy_(nxt.to(tok.device))
        st.pos[m][i] = T
        st.lens[m][i] = T + 1
        self.active[m][i] = 1
        self.host_active[row] = 1
        self.host_len[row] = T + 1
        return tok

    # ------------------------------------------------------------------ decode rounds
    def _set_active(self, active: Sequence[int]):
        """Rows released since the last command go back to position 0 with one key."""
        st = self.st
        for r, a in enumerate(active):
            a = int(a)
            if a == self.host_active[r]:
                continue
            m, i = divmod(r, self.b)
            self.active[m][i] = a
            self.host_active[r] = a
            if not a:
                st.pos[m][i] = 0
                st.lens[m][i] = 1
                self.host_len[r] = 1

    def _decode_body(self, m: int, max_len: int):
        st, b = self.st, self.b
        ctx = AttnCtx("decode", b, 1, st.pos[m], st.lens[m], max_len, st._rows(m), st.rope)
        out = st.model(st.tok[m].view(b, 1) if st.is_first else None, ctx, hidden=None if st.is_first else st.hin[m])
        if st.is_last:
            sp = self.sp
            nxt = ops.sample(out, self.seen[m], sp.temperature, sp.top_k, sp.top_p, sp.repetition_penalty,
                             self.rng[m], sp.do_sample)
            ops.decode_advance(nxt, st.tok[m], self.out[m], self.step_[m], st.pos[m], st.lens[m], self.rng[m],
                               self.active[m])
            return
        st.hout[m].copy_(out)
        st.pos[m].add_(self.active[m])
        st.lens[m].add_(self.active[m])

    @torch.no_grad()
    def step(self, n: int, active: Sequence[int]) -> torch.Tensor:
        """``n`` decode rounds of every row; returns the new tokens [M b, n] (last stage)."""
        st, eng = self.st, self.eng
        M, b, P = self.M, self.b, st.world
        self._set_active(active)
        # the tokens the last stage sampled since the previous round (admissions, the previous
        # command's final round) -> stage 0, which embeds them
        if P > 1 and (st.is_first or st.is_last):
            if st.is_last:
                st._exchange([(torch.stack(st.tok).contiguous(), 0)], [])
            else:
                buf = torch.empty(M, b, dtype=torch.long, device=st.device)
                st._exchange([], [(buf, P - 1)])
                for m in range(M):
                    st.tok[m].copy_(buf[m])
        base = [max(self.host_len[m * b:(m + 1) * b]) for m in range(M)]
        n_items = n * M
        R = st.rank
        for t in range(n_items + P - 1):
            sends, recvs = [], []
            prv, cur = t - 1 - R, t - R
            if P > 1 and 0 <= prv < n_items:
                if not st.is_last:
                    sends.append((st.hout[prv % M], st.next))
                elif prv // M + 1 < n:               # feeds stage 0's next round
                    sends.append((st.tok[prv % M], 0))
            if not st.is_first and 0 <= cur < n_items:
                recvs.append((st.hin[cur % M], st.prev))
            if st.is_first and P > 1:
                prod = t - P                         # item the last stage computed at tick t - 1
                if 0 <= prod < n_items and prod // M + 1 < n:
                    recvs.append((st.tok[prod % M], P - 1))
            st._exchange(sends, recvs)
            if 0 <= cur < n_items:
                k, m = divmod(cur, M)
                self._decode_body(m, min(st.max_seq, base[m] + k))
        for r in range(M * b):
            if self.host_active[r]:
                self.host_len[r] += n
        c0 = self.col
        self.col += n
        if st.is_last:
            return torch.cat([o[:, c0:c0 + n] for o in self.out]).to(eng.cdev)
        return torch.zeros(M * b, n, dtype=torch.long, device=eng.cdev)


def handle_slot_command(eng, hdr0: torch.Tensor) -> None:
    """Worker side of the three slot commands (``serve_workers``); ``hdr0`` = the command header."""
    cmd = int(hdr0[0])
    if cmd == CMD_SLOT_OPEN:
        fl = eng._bcast(torch.zeros(4, dtype=torch.float64, device=eng.cdev))
        sp = _sampling_of(hdr0, fl)
        eng._slot_sess = _SlotSession(eng, sp, int(hdr0[2]), int(hdr0[3])) if eng.member else None
    elif cmd == CMD_SLOT_ADMIT:
        ids = eng._bcast(torch.zeros(int(hdr0[3]), dtype=torch.long, device=eng.cdev))
        tok = eng._slot_sess.admit(int(hdr0[2]), ids) if eng.member else torch.zeros(1, dtype=torch.long,
                                                                                     device=eng.cdev)
        eng._deliver([tok])
    elif cmd == CMD_SLOT_STEP:
        act = eng._bcast(torch.zeros(eng.M * eng.b, dtype=torch.int32, device=eng.cdev))
        n = int(hdr0[2])
        toks = eng._slot_sess.step(n, act.tolist()) if eng.member else \
            torch.zeros(eng.M * eng.b, n, dtype=torch.long, device=eng.cdev)
        eng._deliver([toks])
    else:
        raise RuntimeError(f"unknown slot command {cmd}")


def _sampling_of(hdr: torch.Tensor, fl: torch.Tensor) -> SamplingParams:
    return SamplingParams(max_new_tokens=1, temperature=float(fl[0]), top_k=int(hdr[5]), top_p=float(fl[1]),
                          repetition_penalty=float(fl[2]), do_sample=bool(int(hdr[4])))


@dataclass
class _Slot:
    tag: object
    prompt_len: int
    max_new: int
    eos: Optional[int]
    t0: float
    t_first: float
    tokens: List[int] = field(default_factory=list)


class PipelineSlotDecoder:
    """Driver (rank 0) side: ``engine.continuous.SlotDecoder``'s interface over a
    ``PipelineGenerator`` (see the module docstring).  Slot s lives in pipeline row
    ``(s % M) * b + s // M``, so the occupied rows spread over the micro-batches."""

    def __init__(self, eng, sampling: SamplingParams, seed: int = 0, width: int = 2048,
                 max_batch: Optional[int] = None):
        assert eng.grank == 0 and eng.member, "the driver (rank 0, stage 0) opens slot sessions"
        self.eng, self.sp = eng, sampling
        rows = eng.M * eng.b
        self.B = min(int(max_batch), rows) if max_batch else rows
        self.rows = [(s % eng.M) * eng.b + s // eng.M for s in range(self.B)]
        self.width = width
        self.gen = eng                               # (ServingEngine reads .gen.max_seq through us)
        self.slots: List[Optional[_Slot]] = [None] * self.B
        self.steps = 0
        hdr = torch.zeros(_HDR, dtype=torch.long, device=eng.cdev)
        hdr[0], hdr[1], hdr[2], hdr[3] = CMD_SLOT_OPEN, eng.tag, int(seed), int(width)
        hdr[4], hdr[5] = int(sampling.do_sample), int(sampling.top_k or 0)
        fl = torch.tensor([sampling.temperature, sampling.top_p if sampling.top_p is not None else 1.0,
                           sampling.repetition_penalty, 0.0], dtype=torch.float64, device=eng.cdev)
        eng._bcast(hdr)
        eng._bcast(fl)
        self.sess = _SlotSession(eng, sampling, int(seed), int(width))
        eng._slot_sess = self.sess

    @property
    def col(self) -> int:
        """Output columns used so far (ServingEngine renews a session past half its width)."""
        return self.sess.col

    # ------------------------------------------------------------------ slots
    def free_slots(self) -> List[int]:
        return [s for s, x in enumerate(self.slots) if x is None]

    def busy(self) -> bool:
        return any(x is not None for x in self.slots)

    def can_admit(self, prompt_len: int, max_new: int) -> bool:
        return bool(self.free_slots()) and prompt_len + max_new <= self.eng.max_seq and \
            self.sess.col - 1 + max_new < self.width

    @torch.no_grad()
    def admit(self, ids: Sequence[int], max_new: int, eos: Optional[int] = None, tag=None) -> int:
        assert self.can_admit(len(ids), max_new), "no slot / cache room for this request"
        s = self.free_slots()[0]
        eng = self.eng
        t0 = time.perf_counter()
        hdr = torch.zeros(_HDR, dtype=torch.long, device=eng.cdev)
        hdr[0], hdr[1], hdr[2], hdr[3] = CMD_SLOT_ADMIT, eng.tag, self.rows[s], len(ids)
        eng._bcast(hdr)
        x = eng._bcast(torch.tensor(list(ids), dtype=torch.long, device=eng.cdev))
        tok = self.sess.admit(self.rows[s], x)
        eng._deliver([tok])
        self.slots[s] = _Slot(tag, len(ids), max_new, eos, t0, time.perf_counter(), [int(tok[0])])
        return s

    @torch.no_grad()
    def step(self, n: int = 1) -> int:
        """Up to ``n`` decode rounds of every occupied slot, never past a slot's token budget."""
        live = [x for x in self.slots if x is not None]
        if not live:
            return 0
        n = min(n, min(x.max_new - len(x.tokens) for x in live), self.width - self.sess.col)
        if n <= 0:
            return 0
        eng = self.eng
        act = [0] * (eng.M * eng.b)
        for s, x in enumerate(self.slots):
            if x is not None:
                act[self.rows[s]] = 1
        hdr = torch.zeros(_HDR, dtype=torch.long, device=eng.cdev)
        hdr[0], hdr[1], hdr[2] = CMD_SLOT_STEP, eng.tag, n
        eng._bcast(hdr)
        a = eng._bcast(torch.tensor(act, dtype=torch.int32, device=eng.cdev))
        toks = self.sess.step(n, a.tolist())
        eng._deliver([toks])
        new = toks.tolist()
        for s, x in enumerate(self.slots):
            if x is not None:
                x.tokens.extend(new[self.rows[s]])
        self.steps += n
        return n

    def poll(self) -> List[tuple]:
        """Release finished slots: [(tag, GenerationResult)] (EOS hit or token budget reached)."""
        now = time.perf_counter()
        done = []
        for s, x in enumerate(self.slots):
            if x is None:
                continue
            toks = x.tokens[:x.max_new]
            hit = x.eos is not None and x.eos in toks
            if hit:
                toks = toks[:toks.index(x.eos) + 1]
            if hit or len(x.tokens) >= x.max_new:
                done.append((x.tag, GenerationResult([toks], [x.prompt_len], now - x.t0, x.t_first - x.t0,
                                                     now - x.t_first, [])))
                self.slots[s] = None
        return done
