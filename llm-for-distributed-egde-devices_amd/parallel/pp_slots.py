"""Continuous (iteration-level) batching over the RCCL pipeline.

``PipelineGenerator.generate`` runs a static batch to completion on every stage: a request that
arrives while a long one decodes waits for it, and a short answer holds its rows until the
longest one ends.  The reference's server hands requests to a 10-thread pool and answers each
on its own (Code/gRPC/server.py:14); here the pipeline's ``M x b`` KV rows become SLOTS, as
``engine.continuous.SlotDecoder`` does on one GPU:

* ``PipelineSlotDecoder`` (driver, rank 0) has SlotDecoder's interface (``can_admit`` /
  ``admit`` / ``admit_batch`` / ``step`` / ``poll`` / ``busy``), so ``serve.server.ServingEngine``
  drives either.  Every call is one command broadcast to all ranks (``serve_workers`` runs it on
  theirs).
* ``admit_batch``: every queued request that fits is admitted by ONE command: the prompts are
  prefilled together in one ragged pass (right-padded, per-row last positions) into a scratch
  cache on every stage (hidden states hop stage to stage once for the whole batch), their K/V rows
  are copied into the free slot rows, and the last stage samples every first token in one launch.
* ``step(n)``: n decode rounds of ALL rows through the usual micro-batched tick schedule (rank
  r computes item i = k M + m at tick i + r; hidden states go r -> r + 1, the tokens sampled on
  the last stage come back to stage 0 one exchange later, M >= P keeps that ring full).  Each row
  carries an on-device token budget: a row that reaches it stops advancing (its active flag drops
  inside the decode body, on every stage alike), so ``n`` is not clipped to the shortest
  remaining request — a nearly finished request no longer forces one command per token on all
  the others.  Free rows ride along at position 0 with one key; ``pos`` / ``seq_lens`` advance by
  the active flags (``ops.decode_advance``), so a finished or free row never writes past its slot.
* on the GPU the decode body of each micro-batch (stage forward, and on the last stage the fused
  sampler, the bookkeeping and the budget update) is a HIP graph per (micro-batch, KV-length
  bucket), captured on its second use and replayed afterwards, as ``PipelineStage`` does; the P2P
  exchanges stay outside the graphs.
* a request that hits EOS or its token budget is released by ``poll`` at the next command
  boundary; its row is admitted to the next queued request at once, while the other rows keep
  decoding.

One sampling configuration per session, as SlotDecoder (the fused sampler takes one per launch).
Greedy requests give exactly the tokens of a single-process ``Generator`` run.  The sampling rank
of a slot session is the last stage (its full LM head): the vocabulary-split head of
``PipelineStage`` runs in ``generate`` jobs, not in slot sessions.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch

from .. import ops
from ..engine.generate import GRAPH_BUCKET, GenerationResult, SamplingParams, needs_host_sampler
from ..engine.kv_cache import KVCache
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
        # per row: active flag (pos / lens increments) and the decode rounds it may still take
        self.active = [torch.zeros(self.b, dtype=torch.int32, device=dev) for _ in range(self.M)]
        self.budget = [torch.zeros(self.b, dtype=torch.int32, device=dev) for _ in range(self.M)]
        self.host_active = [0] * (self.M * self.b)
        self.host_budget = [0] * (self.M * self.b)
        self.host_len = [1] * (self.M * self.b)        # keys each row attends over next (upper bound)
        self.col = 1                                   # out column the next decode round writes
        for m in range(self.M):
            st.pos[m].zero_()
            st.lens[m].fill_(1)
            st.tok[m].zero_()
        V = st.cfg.vocab_size
        # vocabulary-split head (parallel/vocab_head.py) when the engine has one and the session's
        # sampling shards: every rank runs its logits slice + sampler phase 1, rank 0 merges and owns
        # the tokens; otherwise the last stage samples with the whole head
        self.vs = vocab_split_session(eng, sampling)
        self.samp = st.is_first if self.vs else st.is_last          # the rank that owns the tokens
        if self.vs or st.is_last:
            Vs = st.shard.Vs if self.vs else V
            self.seen = [torch.zeros(self.b, Vs, dtype=torch.uint8, device=dev) for _ in range(self.M)]
            self.rng = [torch.tensor([(seed + 7919 * m) & 0x7FFFFFFF, 1], dtype=torch.int32, device=dev)
                        for m in range(self.M)]
        if st.is_last:
            self.rng_adm = torch.tensor([(seed + 104729) & 0x7FFFFFFF, 0], dtype=torch.int32, device=dev)
        if self.samp:
            self.step_ = [torch.ones(1, dtype=torch.long, device=dev) for _ in range(self.M)]
            self.out = [torch.zeros(self.b, width, dtype=torch.long, device=dev) for _ in range(self.M)]
        if self.vs:
            P = st.world
            mode = ops.shard_mode(sampling.temperature, sampling.top_k, sampling.top_p, V, sampling.do_sample)
            self.hfin = [torch.zeros(self.b, st.cfg.hidden_size, dtype=st.model.dtype, device=dev)
                         for _ in range(self.M)]
            self.cand: Dict[int, tuple] = {}
            if st.is_first:
                vb = st.vs_bounds
                self.cand_in = [[tuple(torch.empty(shp, dtype=dt, device=dev) for shp, dt in
                                       ops.shard_candidate_shapes(self.b, vb[r + 1] - vb[r], V, mode, dev))
                                 for r in range(1, P)] for _ in range(self.M)]
            else:
                self.tokin = [torch.zeros(self.b, dtype=torch.long, device=dev) for _ in range(self.M)]
        # decode graphs per (micro-batch, KV bucket): GPU, a sampler that stays on the device
        self.use_graphs = bool(st.use_graphs and st.cuda and getattr(st.kv, "graph_safe", True)
                               and not needs_host_sampler(sampling, st.cfg.vocab_size)
                               and all(getattr(mm, "graph_safe", True) or getattr(mm, "graph_safe_rows", 0) >= self.b
                                       for mm in st.model.modules()))
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self._warm: Dict[int, bool] = {}
        self._pool = None

    # ------------------------------------------------------------------ admission
    @torch.no_grad()
    def admit_batch(self, rows: Sequence[int], lens: Sequence[int], max_new: Sequence[int],
                    ids_cat: torch.Tensor) -> torch.Tensor:
        """Prefill k prompts (concatenated in ``ids_cat``, lengths ``lens``) into ``rows`` on this
        stage in ONE ragged pass; the last stage samples every first token in one launch.  Returns
        the k first tokens (meaningful on the last stage)."""
        st, eng = self.st, self.eng
        k = len(rows)
        dev = st.device
        H = st.cfg.hidden_size
        T = max(lens)
        lens_t = torch.tensor(list(lens), dtype=torch.long)
        # [k, T] right-padded; a pad repeats its row's first token (never a new penalty id)
        ids = torch.empty(k, T, dtype=torch.long)
        off = 0
        flat = ids_cat.to("cpu", torch.long)
        for i, n in enumerate(lens):
            ids[i, :n] = flat[off:off + n]
            ids[i, n:] = flat[off]
            off += n
        ids = ids.to(dev)
        r0 = min(rows)
        direct = sorted(rows) == list(range(r0, r0 + k))   # contiguous slot rows: prefill in place
        scratch = None if direct else KVCache(st.cfg, k, T, st.kv.first, st.kv.last, st.model.dtype, dev,
                                              kv_dtype=st.kv_dtype, zero=False)   # every row written [0, T)
        order = sorted(range(k), key=lambda i: rows[i]) if direct else list(range(k))
        if direct and order != list(range(k)):          # rows in cache order
            rows, lens, max_new = [rows[i] for i in order], [lens[i] for i in order], [max_new[i] for i in order]
            ids, lens_t = ids[order], lens_t[order]
        sp0 = torch.zeros(k, dtype=torch.int32, device=dev)
        last = (lens_t - 1).to(dev)
        view = st.kv.rows(r0, r0 + k) if direct else scratch.rows(0, k)
        ctx = AttnCtx("prefill", k, T, sp0, sp0 + T, T, view, st.rope, last_pos=last)
        hidden = None
        if not st.is_first:
            hidden = torch.empty(k * T, H, dtype=st.model.dtype, device=dev)
            st._exchange([], [(hidden, st.prev)])
        out = st.model(ids if st.is_first else None, ctx, hidden=hidden, logits="last")
        if not st.is_last:
            st._exchange([(out.contiguous(), st.next)], [])
        if scratch is not None:
            # the prompt's K / V rows into the slot rows of the session's cache (one copy per tensor)
            ridx = torch.tensor(list(rows), dtype=torch.long, device=dev)
            for name in ("k", "v") + (("ks", "vs") if scratch.quantized else ()):
                dst, src = getattr(st.kv, name), getattr(scratch, name)
                dst[:, ridx, :, :T] = src
            del scratch
        toks = torch.zeros(k, dtype=torch.long, device=eng.cdev)
        mb = [divmod(r, self.b) for r in rows]
        nxt = None
        if st.is_last:                                 # the first tokens: the last stage's whole head
            seen = torch.zeros(k, st.cfg.vocab_size, dtype=torch.uint8, device=dev)
            seen.scatter_(1, ids, 1)
            sp = self.sp
            nxt = ops.sample(out, seen, sp.temperature, sp.top_k, sp.top_p, sp.repetition_penalty, self.rng_adm,
                             sp.do_sample)
            self.rng_adm[1:].add_(1)
            if not self.vs:
                for i, (m, j) in enumerate(mb):
                    self.seen[m][j].copy_(seen[i])
        if self.vs:
            # the first tokens -> every rank: each marks the prompt and the token in its shard of the
            # penalty flags, rank 0 (which merges from now on) keeps them as the rows' tokens
            P = st.world
            if st.is_last:
                st._exchange([(nxt, r) for r in range(P - 1)], [])
            else:
                nxt = torch.empty(k, dtype=torch.long, device=dev)
                st._exchange([], [(nxt, P - 1)])
            for i, (m, j) in enumerate(mb):
                row = torch.zeros(1, self.seen[m].shape[1], dtype=torch.uint8, device=dev)
                for t in (ids[i], nxt[i:i + 1]):
                    jj = t.view(-1) - st.shard.v0
                    jj = jj[(jj >= 0) & (jj < row.shape[1])]
                    row[0, jj] = 1
                self.seen[m][j:j + 1].copy_(row)
        if self.samp:
            for i, (m, j) in enumerate(mb):
                st.tok[m][j:j + 1].copy_(nxt[i:i + 1])
                self.out[m][j].zero_()
                self.out[m][j, self.col - 1:self.col].copy_(nxt[i:i + 1])
            toks[torch.tensor(order, device=toks.device)] = nxt.to(toks.device)   # the caller's order
        for i, (m, j) in enumerate(mb):
            n = int(lens[i])
            b_left = max(0, int(max_new[i]) - 1)        # the first token came from the prefill
            st.pos[m][j] = n
            st.lens[m][j] = n + 1
            self.active[m][j] = 1 if b_left > 0 else 0
            self.budget[m][j] = b_left
            r = rows[i]
            self.host_active[r] = 1 if b_left > 0 else 0
            self.host_budget[r] = b_left
            self.host_len[r] = n + 1
        return toks

    # ------------------------------------------------------------------ decode rounds
    def _release(self, released: Sequence[int]):
        """Rows the driver released since the last command go back to position 0 with one key."""
        st = self.st
        for r in released:
            m, i = divmod(int(r), self.b)
            self.active[m][i] = 0
            self.budget[m][i] = 0
            st.pos[m][i] = 0
            st.lens[m][i] = 1
            self.host_active[r] = 0
            self.host_budget[r] = 0
            self.host_len[r] = 1

    def _decode_body(self, m: int, max_len: int):
        st, b = self.st, self.b
        ctx = AttnCtx("decode", b, 1, st.pos[m], st.lens[m], max_len, st._rows(m), st.rope)
        out = st.model(st.tok[m].view(b, 1) if st.is_first else None, ctx, hidden=None if st.is_first else st.hin[m],
                       logits="hidden" if self.vs else "last")
        if st.is_last and self.vs:                    # the final-normed rows go to every rank's head shard
            self.hfin[m].copy_(out)
            st.pos[m].add_(self.active[m])
            st.lens[m].add_(self.active[m])
        elif st.is_last:
            sp = self.sp
            nxt = ops.sample(out, self.seen[m], sp.temperature, sp.top_k, sp.top_p, sp.repetition_penalty,
                             self.rng[m], sp.do_sample)
            ops.decode_advance(nxt, st.tok[m], self.out[m], self.step_[m], st.pos[m], st.lens[m], self.rng[m],
                               self.active[m])
        else:
            st.hout[m].copy_(out)
            st.pos[m].add_(self.active[m])
            st.lens[m].add_(self.active[m])
        # every stage alike: a row that used its last round stops advancing
        self.budget[m].sub_(self.active[m])
        self.active[m].mul_(self.budget[m].gt(0).to(torch.int32))

    def _bucket(self, n: int) -> int:
        return min(self.st.max_seq, ((n + GRAPH_BUCKET - 1) // GRAPH_BUCKET) * GRAPH_BUCKET)

    def _decode(self, m: int, max_len: int):
        if not self.use_graphs:
            return self._decode_body(m, max_len)
        bucket = self._bucket(max_len)
        if not self._warm.get(m):
            self._warm[m] = True
            return self._decode_body(m, bucket)         # first decode of m: eager (warm-up)
        g = self._graphs.get((m, bucket))
        if g is None:
            # every P2P of this tick has completed on the host's order (``_exchange``), and capture
            # records without executing: the device is idle before the capture starts
            torch.cuda.synchronize(self.st.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self._pool, capture_error_mode="thread_local"):
                self._decode_body(m, bucket)
            if self._pool is None:
                self._pool = g.pool()
            self._graphs[(m, bucket)] = g
        g.replay()

    # ---------------------------------------------------------- vocabulary-split head (self.vs)
    def _vs_shard(self, m: int):
        """This rank's logits slice + sampler phase 1 for the rows of micro-batch m (in hfin[m])."""
        st = self.st
        self.cand[m] = st.shard.candidates(self.hfin[m], self.seen[m], self.sp, self.rng[m])
        if not st.is_first:
            self.rng[m][1:].add_(1)                   # rank 0 advances after its merge (same step)

    def _vs_merge(self, m: int):
        """Rank 0: phase 2 over every shard's candidates -> the token of each row of m, and the
        decode bookkeeping of the sampling rank (out column, step, noise counter, penalty flags)."""
        st, sp = self.st, self.sp
        nxt = ops.sample_merge([self.cand[m]] + self.cand_in[m], st.cfg.vocab_size, sp.temperature, sp.top_k,
                               sp.top_p, self.rng[m], sp.do_sample)
        st.tok[m].copy_(nxt)
        self.out[m].scatter_(1, self.step_[m].view(1, 1).expand(self.b, 1), nxt.view(self.b, 1))
        self.rng[m][1:].add_(1)
        self.step_[m].add_(1)
        ops.seen_mark(self.seen[m], nxt, st.shard.v0)

    @torch.no_grad()
    def _step_vs(self, n: int) -> torch.Tensor:
        """``n`` decode rounds with the vocabulary-split head.  Item i = k M + m runs on rank r at
        tick i + r; its final-normed rows leave the last stage at tick i + P, every rank runs its
        head shard then, rank 0 merges at i + P + 1 (the token item i + M embeds, M >= P + 1) and
        sends it on at i + P + 2, when the other ranks mark it in their penalty shards.  The loop
        drains every stage of the command's last round before it returns."""
        st = self.st
        M, b, P, R = self.M, self.b, st.world, st.rank
        assert M >= P + 1, "the vocab-split head needs >= P + 1 micro-batches"
        base = [max(self.host_len[m * b:(m + 1) * b]) for m in range(M)]
        n_items = n * M
        valid = lambda i: 0 <= i < n_items              # noqa: E731
        for t in range(n_items + P + 2):
            sends, recvs = [], []
            prv, cur = t - 1 - R, t - R
            if valid(prv) and not st.is_last:
                sends.append((st.hout[prv % M], st.next))
            if valid(cur) and not st.is_first:
                recvs.append((st.hin[cur % M], st.prev))
            # (after the hand-offs: P2P ops of a rank pair match in posting order)
            hg, cg, mg = t - P, t - P - 1, t - P - 2
            if valid(hg):
                if st.is_last:
                    sends.extend((self.hfin[hg % M], r) for r in range(P - 1))
                else:
                    recvs.append((self.hfin[hg % M], P - 1))
            if valid(cg):
                if st.is_first:
                    recvs.extend((x, r + 1) for r, c in enumerate(self.cand_in[cg % M]) for x in c)
                else:
                    sends.extend((x, 0) for x in self.cand[cg % M])
            if valid(mg):
                if st.is_first:
                    sends.extend((st.tok[mg % M], r) for r in range(1, P))
                else:
                    recvs.append((self.tokin[mg % M], 0))
            st._exchange(sends, recvs)
            if valid(mg) and not st.is_first:
                ops.seen_mark(self.seen[mg % M], self.tokin[mg % M], st.shard.v0)
            if valid(cg) and st.is_first:
                self._vs_merge(cg % M)
            if valid(hg):
                self._vs_shard(hg % M)
            if valid(cur):
                k, m = divmod(cur, M)
                self._decode(m, min(st.max_seq, base[m] + k))
        self._advance_host(n)
        c0 = self.col
        self.col += n
        if st.is_first:
            return torch.cat([o[:, c0:c0 + n] for o in self.out]).to(self.eng.cdev)
        return torch.zeros(M * b, n, dtype=torch.long, device=self.eng.cdev)

    def _advance_host(self, n: int):
        for r in range(self.M * self.b):
            if self.host_active[r]:
                used = min(n, self.host_budget[r])
                self.host_len[r] += used
                self.host_budget[r] -= used
                if self.host_budget[r] == 0:
                    self.host_active[r] = 0

    @torch.no_grad()
    def step(self, n: int, released: Sequence[int]) -> torch.Tensor:
        """``n`` decode rounds of every row; returns the new tokens [M b, n] (on the sampling rank:
        the last stage, or rank 0 under the vocabulary-split head)."""
        st, eng = self.st, self.eng
        M, b, P = self.M, self.b, st.world
        self._release(released)
        if self.vs:
            return self._step_vs(n)
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
                self._decode(m, min(st.max_seq, base[m] + k))
        self._advance_host(n)
        c0 = self.col
        self.col += n
        if st.is_last:
            return torch.cat([o[:, c0:c0 + n] for o in self.out]).to(eng.cdev)
        return torch.zeros(M * b, n, dtype=torch.long, device=eng.cdev)


def vocab_split_session(eng, sampling: SamplingParams) -> bool:
    """Whether a slot session of ``eng`` samples with the vocabulary-split head (every rank derives
    it alike from the engine and the session's sampling configuration)."""
    return bool(getattr(eng, "vs_req", False) and eng.world > 1 and
                ops.shard_mode(sampling.temperature, sampling.top_k, sampling.top_p, eng.cfg.vocab_size,
                               sampling.do_sample) >= 0)


def handle_slot_command(eng, hdr0: torch.Tensor) -> None:
    """Worker side of the three slot commands (``serve_workers``); ``hdr0`` = the command header."""
    cmd = int(hdr0[0])
    if cmd == CMD_SLOT_OPEN:
        fl = eng._bcast(torch.zeros(4, dtype=torch.float64, device=eng.cdev))
        sp = _sampling_of(hdr0, fl)
        eng._slot_sess = _SlotSession(eng, sp, int(hdr0[2]), int(hdr0[3])) if eng.member else None
        eng._slot_res = 0 if vocab_split_session(eng, sp) else eng.world - 1   # stage holding the tokens
    elif cmd == CMD_SLOT_ADMIT:
        k, total = int(hdr0[2]), int(hdr0[3])
        meta = eng._bcast(torch.zeros(k, 3, dtype=torch.long, device=eng.cdev))
        ids = eng._bcast(torch.zeros(total, dtype=torch.long, device=eng.cdev))
        if eng.member:
            mt = meta.tolist()
            toks = eng._slot_sess.admit_batch([x[0] for x in mt], [x[1] for x in mt], [x[2] for x in mt], ids)
        else:
            toks = torch.zeros(k, dtype=torch.long, device=eng.cdev)
        eng._deliver([toks], eng._slot_res)
    elif cmd == CMD_SLOT_STEP:
        nrel = int(hdr0[3])
        rel = eng._bcast(torch.zeros(max(1, nrel), dtype=torch.int32, device=eng.cdev))
        n = int(hdr0[2])
        toks = eng._slot_sess.step(n, rel.tolist()[:nrel]) if eng.member else \
            torch.zeros(eng.M * eng.b, n, dtype=torch.long, device=eng.cdev)
        eng._deliver([toks], eng._slot_res)
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
        self._released: List[int] = []               # rows freed by poll, reset on the next command
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
        eng._slot_res = 0 if self.sess.vs else eng.world - 1

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
        return self.admit_batch([(ids, max_new, eos, tag)])[0]

    @torch.no_grad()
    def admit_batch(self, reqs: Sequence[tuple]) -> List[int]:
        """Admit ``reqs`` = [(ids, max_new, eos, tag)] with ONE command (one ragged prefill on every
        stage, one sampler launch); returns their slots."""
        free = self.free_slots()
        assert len(reqs) <= len(free), "more requests than free slots"
        for ids, mx, _, _ in reqs:
            assert self.can_admit(len(ids), mx), "no slot / cache room for this request"
        eng = self.eng
        t0 = time.perf_counter()
        slots = free[:len(reqs)]
        k = len(reqs)
        meta = torch.tensor([[self.rows[s], len(r[0]), int(r[1])] for s, r in zip(slots, reqs)], dtype=torch.long,
                            device=eng.cdev)
        cat = [int(t) for r in reqs for t in r[0]]
        hdr = torch.zeros(_HDR, dtype=torch.long, device=eng.cdev)
        hdr[0], hdr[1], hdr[2], hdr[3] = CMD_SLOT_ADMIT, eng.tag, k, len(cat)
        eng._bcast(hdr)
        eng._bcast(meta)
        x = eng._bcast(torch.tensor(cat, dtype=torch.long, device=eng.cdev))
        self._flush_released()
        toks = self.sess.admit_batch([self.rows[s] for s in slots], [len(r[0]) for r in reqs],
                                     [int(r[1]) for r in reqs], x)
        eng._deliver([toks], eng._slot_res)
        first = toks.tolist()
        t1 = time.perf_counter()
        for s, r, tk in zip(slots, reqs, first):
            ids, mx, eos, tag = r
            self.slots[s] = _Slot(tag, len(ids), mx, eos, t0, t1, [int(tk)])
        return slots

    def _flush_released(self):
        """Released rows are reset by the workers with the next STEP command; an admission reuses
        a row directly (its prefill rewrites the row's whole state), so it is dropped from the list."""
        taken = set(self.rows[s] for s, x in enumerate(self.slots) if x is not None)
        self._released = [r for r in self._released if r not in taken]

    @torch.no_grad()
    def step(self, n: int = 1) -> int:
        """``n`` decode rounds of every occupied slot (each row stops on the device at its token
        budget, so the round count is not clipped to the shortest remaining request)."""
        live = [x for x in self.slots if x is not None and len(x.tokens) < x.max_new]
        if not live:
            return 0
        n = min(n, max(x.max_new - len(x.tokens) for x in live), self.width - self.sess.col)
        if n <= 0:
            return 0
        eng = self.eng
        self._flush_released()
        rel = list(self._released)
        self._released = []
        hdr = torch.zeros(_HDR, dtype=torch.long, device=eng.cdev)
        hdr[0], hdr[1], hdr[2], hdr[3] = CMD_SLOT_STEP, eng.tag, n, len(rel)
        eng._bcast(hdr)
        r = eng._bcast(torch.tensor(rel or [0], dtype=torch.int32, device=eng.cdev))
        toks = self.sess.step(n, r.tolist()[:len(rel)])
        eng._deliver([toks], eng._slot_res)
        new = toks.tolist()
        for s, x in enumerate(self.slots):
            if x is not None:
                x.tokens.extend(new[self.rows[s]][:max(0, x.max_new - len(x.tokens))])
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
                self._released.append(self.rows[s])
        return done
