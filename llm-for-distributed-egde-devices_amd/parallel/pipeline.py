"""Layer-partitioned inference pipeline: one process per GPU ("edge device"), RCCL P2P over xGMI.

The reference only ever splits a model implicitly through accelerate's ``device_map="auto"``
(activations hop GPUs via ``tensor.to(next_device)``, no micro-batching — SURVEY §2.4, K16;
Code/Base Models/Llama_bf16_updated.py:31) and ships no tensors over its gRPC demo.  Here every
stage is its own process; hidden states move rank r -> r+1 with RCCL point-to-point, and the
tokens sampled on the last stage travel back to stage 0 (a token ring), so decode keeps every
stage busy:

  work items (same order on every rank):  prefill(m) for m < M, then decode(k, m) for k < S
  rank s processes item i at tick i + s (lockstep); with M >= P micro-batches the token of
  decode(k, m) reaches stage 0 exactly when decode(k+1, m) starts (M - P ticks of slack).

Per tick each rank issues one grouped P2P exchange per lane through ``dist.batch_isend_irecv``
(send the lane's previous outputs, receive its next inputs — grouped, so no send/recv ordering
deadlock; on RCCL one ncclGroupStart/End), issued and completed on that lane's HIP stream, then
runs its layers for the micro-batches of the tick.  By default all lanes share the stage group's
communicator: each lane posts and completes its exchange on its own stream, and RCCL runs the
lanes' hops one after another on its internal stream.  ``EDGELLM_LANE_GROUPS=1`` gives every lane
its OWN process group (``lane_groups``; one RCCL communicator, hence one more internal stream, per
lane), so a lane's hop waits only for that lane's compute.  It is opt-in: a process
has GPU_MAX_HW_QUEUES = 4 hardware queues, and default + 2 lane streams + 3 communicator streams
would share them, putting a spinning RCCL receive kernel in front of another stream's compute on
one queue — a cross-rank dependency cycle; with one communicator the streams fit the queues.
(Measured under gloo — the 2 / 4 / 8-rank rehearsals — and at RCCL world 1; the multi-GPU RCCL
overlap is unmeasured.)  The same P2POp path runs under gloo on the CPU, which is how the
multi-rank schedule is tested without GPUs.  The decode compute of each micro-batch is captured in
a HIP graph per KV-length bucket (all buckets of a run are captured at the first capture, before
any timed region); the P2P ops stay outside the graphs on RCCL's stream, ordered by stream waits,
so the host never blocks on the device inside the loop.  Messages: decode b*H*2 bytes per hop
(128 x 4096 bf16 = 1 MiB), prefill b*T*H*2.

Communicator set-up is eager: ``init_distributed`` binds the rank's device (``device_id``) so
RCCL builds the world communicator at init, and ``PipelineStage.__init__`` runs one all-ranks
collective before any P2P (``batch_isend_irecv`` requires the first op on a communicator to be
joined by every rank).  Per-tick device events give every rank's compute time, P2P wait and
bubble fraction over a window of ticks (``run(stats_window=...)`` -> ``PipelineResult.stats``).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import ops
from ..engine.generate import GRAPH_BUCKET, SamplingParams, needs_host_sampler
from ..engine.kv_cache import KVCache, resolve_kv_dtype
from ..models.decoder import AttnCtx, DecoderLM
from ..utils.tracing import debug_sync, trace_range


@dataclass
class PipelineResult:
    tokens: Optional[List[List[int]]]    # last rank: generated ids per sequence (micro-batch major)
    ticks: int
    elapsed_s: float
    marks: Dict[str, float] = field(default_factory=dict)
    stats: Dict[str, float] = field(default_factory=dict)   # this rank, over the stats window


class PipelineStage:
    def __init__(self, model: DecoderLM, rank: int, world: int, micro_batch: int, n_micro: int, max_seq: int,
                 group=None, use_graphs: Optional[bool] = None, headinfer_heads: Optional[int] = None,
                 lanes: int = 1, prefill_chunk: int = 4096, warm_comm: bool = True, kv_dtype: str = "bf16",
                 ranks: Optional[Sequence[int]] = None, slack: int = 0, vocab_split: bool = False,
                 head_shard=None):
        """``headinfer_heads``: keep only this many KV heads per layer on the GPU and offload the rest
        to pinned host memory (edgellm.offload.HeadInferKV; BASELINE config "8-way pipeline +
        HeadInfer").  The offloaded path is host-orchestrated on one compute stream, so it runs one
        lane and its decode steps run eagerly; its cache is built at ``run`` with prefill chunks
        of min(prompt_len, ``prefill_chunk``) tokens and staging buffers of one micro-batch.

        ``rank`` / ``world`` are the stage index and stage count within ``group``; ``ranks`` maps
        stage index -> global rank (default identity: the stages are ranks 0..world-1), so a model
        can be pipelined over any rank subset (one ``dist.new_group`` per ensemble agent).

        ``vocab_split`` (world > 1): the LM head is split by vocabulary over every rank
        (parallel/vocab_head.py; ``head_shard`` = this rank's rows): the last stage hands its
        final-normed hidden rows to every rank, each rank runs its logits slice + sampler phase 1,
        rank 0 merges (phase 2), owns the sampled tokens and sends them to the other ranks for their
        repetition-penalty flags.  Needs D (P + 1) micro-batch groups in flight (D = 1 + slack); runs
        whenever the sampling configuration shards (ops.shard_mode), else the last stage samples."""
        assert lanes >= 1 and n_micro % lanes == 0, "micro-batches must split evenly over lanes"
        assert n_micro >= world * lanes, "need lanes x stages micro-batches to keep the ring full"
        offload = headinfer_heads is not None and headinfer_heads < model.cfg.num_kv_heads
        assert not offload or lanes == 1, "HeadInfer offload orders its transfers on one stream: use lanes=1"
        self.model, self.cfg = model, model.cfg
        self.rank, self.world = rank, world
        self.b, self.M = micro_batch, n_micro
        self.max_seq = max_seq
        self.group = group
        self.device = model.device
        # KV layers: the stage's layers with an attention half (a stage opening on an MLP half has none for it)
        self.first, self.last = getattr(model, "kv_first", model.first), model.last
        self.is_first, self.is_last = model.has_embed, model.has_head
        assert self.is_first == (rank == 0) and self.is_last == (rank == world - 1)
        self.prev = (rank - 1) % world
        self.next = (rank + 1) % world
        self.slack = int(slack)                       # extra ticks per hop (P2P overlapped with compute)
        self.granks = list(ranks) if ranks is not None else list(range(world))
        assert len(self.granks) == world, "one global rank per stage"
        self.h_on = headinfer_heads if offload else None
        self.prefill_chunk = max(1, prefill_chunk)
        self.kv_dtype = kv_dtype = resolve_kv_dtype(kv_dtype, self.cfg, model.dtype, self.device)
        self.kv = None if offload else KVCache(self.cfg, micro_batch * n_micro, max_seq, self.first, self.last,
                                               model.dtype, self.device, kv_dtype=kv_dtype)
        self.attn_hook = None
        self.rope = model.rope_table(self.device)
        cuda = self.device.type == "cuda"
        self.cuda = cuda
        self.use_graphs = cuda if use_graphs is None else (use_graphs and cuda)
        self.nccl = dist.is_initialized() and dist.get_backend(group) == "nccl"
        # gloo with device tensors (several ranks sharing one GPU for a rehearsal): P2P is staged
        # through host memory
        self.host_staged = cuda and dist.is_initialized() and not self.nccl
        H, b, dev = self.cfg.hidden_size, micro_batch, self.device
        self.tok = [torch.zeros(b, dtype=torch.long, device=dev) for _ in range(n_micro)]
        self.pos = [torch.zeros(b, dtype=torch.int32, device=dev) for _ in range(n_micro)]
        self.lens = [torch.ones(b, dtype=torch.int32, device=dev) for _ in range(n_micro)]
        self.hin = [torch.zeros(b, H, dtype=model.dtype, device=dev) for _ in range(n_micro)]
        self.hout = [torch.zeros(b, H, dtype=model.dtype, device=dev) for _ in range(n_micro)]
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self._pools: Dict[int, object] = {}
        # lanes: micro-batches m with equal m % lanes share a HIP stream and a graph memory pool;
        # the lanes of a tick run concurrently (their graphs never share intermediate buffers)
        self.L = lanes
        self.streams = ([torch.cuda.Stream(self.device) for _ in range(lanes)]
                        if cuda and lanes > 1 else None)
        self.p2p_bytes = 0
        self._copy_stream = None                      # host-staged sends (gloo with device tensors)
        self._plen, self._eos = None, None            # per-run: ragged prompt lengths, EOS id (last rank)
        # EDGELLM_LANE_GROUPS=1: one process group (communicator) per lane for the per-lane exchanges
        # (lanes > 1 on GPU streams; only the stage ranks join its creation: use_local_synchronization)
        self.lane_groups = [group] * lanes
        import os
        if (self.streams is not None and dist.is_initialized() and world > 1
                and os.environ.get("EDGELLM_LANE_GROUPS", "0") == "1"):
            self.lane_groups = [dist.new_group(self.granks, use_local_synchronization=True) for _ in range(lanes)]
        self.vs_req = bool(vocab_split) and world > 1
        self.shard = head_shard
        self.vs = False                               # per run: vocab split active
        if self.vs_req:
            from .vocab_head import shard_bounds
            assert head_shard is not None, "vocab_split needs this rank's head shard"
            self.vs_bounds = shard_bounds(self.cfg.vocab_size, world)
            assert (head_shard.v0, head_shard.v1) == (self.vs_bounds[rank], self.vs_bounds[rank + 1]), \
                "head shard rows do not match vocab_head.shard_bounds"
        if warm_comm and dist.is_initialized() and world > 1:
            self.warm_communicator()

    def warm_communicator(self):
        """One collective every rank joins: creates RCCL's world communicator (and its xGMI peer
        connections' first use) before the first grouped P2P, outside any timed region."""
        x = torch.ones(1, device=self.device if self.nccl else "cpu")
        dist.all_reduce(x, group=self.group)
        for g in self.lane_groups:
            if g is not self.group:
                dist.all_reduce(x, group=g)
        if self.cuda:
            torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ p2p
    def _exchange(self, sends, recvs):
        """sends/recvs: lists of (tensor, peer stage).  One grouped exchange (dist.P2POp batch),
        completed before returning (the current stream waits on it; host-staged: the host)."""
        self._finish(self._post(sends, recvs))

    def _post(self, sends, recvs, send_ready=None, group=None):
        """Issue one grouped exchange without waiting for it; ``_finish`` completes it.  RCCL: the
        communication stream first waits on everything already queued on the current stream (the
        sends' producers), so posting BEFORE the next compute lets the transfer run beside it.
        Host-staged (gloo with device tensors): the sends are copied to pinned host memory on a side
        stream behind ``send_ready`` (an event after their producer), so the host never waits for
        compute queued after it; received bytes land in pinned buffers until ``_finish``."""
        if not sends and not recvs:
            return None
        self.p2p_bytes += sum(t.numel() * t.element_size() for t, _ in sends)
        g = self.granks
        pg = self.group if group is None else group
        if self.host_staged:
            if self._copy_stream is None:
                self._copy_stream = torch.cuda.Stream(self.device)
            cs = self._copy_stream
            producer = torch.cuda.current_stream(self.device)   # (taken before cs becomes current)
            assert producer != cs, "the copy stream must wait on the sends' producer, not on itself"
            host_sends = []
            with torch.cuda.stream(cs):
                if send_ready is not None:
                    cs.wait_event(send_ready)
                else:
                    cs.wait_stream(producer)
                for t, _ in sends:
                    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                    h.copy_(t, non_blocking=True)
                    host_sends.append(h)
            cs.synchronize()
            bufs = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t, _ in recvs]
            p2p = [dist.P2POp(dist.isend, h, g[p], pg) for h, (_, p) in zip(host_sends, sends)]
            p2p += [dist.P2POp(dist.irecv, h, g[p], pg) for h, (_, p) in zip(bufs, recvs)]
        else:
            bufs = None
            p2p = [dist.P2POp(dist.isend, t, g[p], pg) for t, p in sends]
            p2p += [dist.P2POp(dist.irecv, t, g[p], pg) for t, p in recvs]
        with trace_range("pp.exchange"):
            works = dist.batch_isend_irecv(p2p)
        return works, bufs, [t for t, _ in recvs], p2p

    def _finish(self, handle):
        """Complete a posted exchange: RCCL — the current stream waits on it (no host block);
        host-staged — the host waits, then the received bytes go to the device on the current
        stream (ordered before the compute that reads them)."""
        if handle is None:
            return
        works, bufs, dsts, _ = handle
        for w in works:
            w.wait()
        if bufs is not None:
            for h, t in zip(bufs, dsts):
                t.copy_(h, non_blocking=True)
        debug_sync("pp.exchange")

    def _send_one(self, t: torch.Tensor, peer: int):
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, self.granks[peer], self.group)]):
            w.wait()

    def _recv_one(self, t: torch.Tensor, peer: int):
        for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, t, self.granks[peer], self.group)]):
            w.wait()

    # ------------------------------------------------------------------ compute
    def _rows(self, m):
        return self.kv.rows(m * self.b, (m + 1) * self.b)

    def _build_offload_kv(self, T: int):
        from ..offload import HeadInferKV
        chunk = min(T, self.prefill_chunk)
        kv = self.kv
        if kv is None or kv.chunk_size != chunk:
            self.kv = None
            if self.cuda:
                torch.cuda.empty_cache()
            self.kv = HeadInferKV(self.cfg, self.b * self.M, self.max_seq, self.h_on, self.device, self.first,
                                  self.last, chunk_size=chunk, dtype=self.model.dtype, call_rows=self.b,
                                  kv_dtype=self.kv_dtype)
        self.attn_hook = self.kv.attn_hook

    def _prefill(self, m: int, ids: Optional[torch.Tensor], T: int, hidden: Optional[torch.Tensor]):
        """Prefill micro-batch m (prompt length T); chunked by ``prefill_chunk`` when the KV is
        offloaded (HeadInfer bounds activation memory by the chunk, as in the paper).  Ragged
        prompts (``self._plen[m]``, right-padded to T) take one pass with per-row last positions."""
        b, H = self.b, self.cfg.hidden_size
        plen = self._plen[m] if self._plen is not None else None
        C = getattr(self.kv, "chunk_size", T) if self.attn_hook is not None else T
        assert plen is None or C >= T, "HeadInfer's chunked prefill takes equal-length prompts"
        outs = []
        out = None
        for c0 in range(0, T, C):
            c1 = min(T, c0 + C)
            sp = torch.full((b,), c0, dtype=torch.int32, device=self.device)
            ctx = AttnCtx("prefill", b, c1 - c0, sp, sp + (c1 - c0), c1, self._rows(m), self.rope,
                          attn_hook=self.attn_hook, last_pos=(plen - 1) if plen is not None else None)
            x_ids = ids[:, c0:c1] if ids is not None else None
            x_h = None
            if hidden is not None:
                x_h = hidden.view(b, T, H)[:, c0:c1].contiguous().view(b * (c1 - c0), H) if C < T else hidden
            out = self.model(x_ids, ctx, hidden=x_h, logits="hidden" if self.vs else "last")
            if not self.is_last and C < T:
                outs.append(out.view(b, c1 - c0, H))
        if outs:
            out = torch.cat(outs, 1).reshape(b * T, H)
        if plen is not None:
            self.pos[m].copy_(plen)
            self.lens[m].copy_(plen + 1)
        else:
            self.pos[m].fill_(T)
            self.lens[m].fill_(T + 1)
        return out

    def _decode_body(self, m: int, max_len: int):
        b = self.b
        ctx = AttnCtx("decode", b, 1, self.pos[m], self.lens[m], max_len, self._rows(m), self.rope,
                      attn_hook=self.attn_hook)
        out = self.model(self.tok[m].view(b, 1) if self.is_first else None, ctx,
                         hidden=None if self.is_first else self.hin[m],
                         logits="hidden" if self.vs else "last")
        if self.is_last and self.vs:                  # vocab split: the final-normed rows go to every rank
            self.hfin[m].copy_(out)
            self.pos[m].add_(1)
            self.lens[m].add_(1)
            return
        if self.is_last:                              # sampler + bookkeeping (pos / lens += 1 included)
            sp = self.sampling
            nxt = ops.sample_advance(out, self.seen[m], sp.temperature, sp.top_k, sp.top_p, sp.repetition_penalty,
                                     self.rng[m], self.tok[m], self.out[m], self.step[m], self.pos[m], self.lens[m],
                                     self.ctr[m], sp.do_sample)
            if self._eos is not None:
                self.hit[m].logical_or_(nxt.eq(self._eos))
            return
        self.hout[m].copy_(out)
        self.pos[m].add_(1)
        self.lens[m].add_(1)

    def _sample(self, m, logits):
        sp = self.sampling
        nxt = ops.sample(logits, self.seen[m], sp.temperature, sp.top_k, sp.top_p, sp.repetition_penalty,
                         self.rng[m], sp.do_sample)
        self.tok[m].copy_(nxt)
        self.out[m].scatter_(1, self.step[m].view(1, 1).expand(self.b, 1), nxt.view(self.b, 1))
        self.rng[m][1:].add_(1)
        self.step[m].add_(1)
        if self._eos is not None:                     # device-side EOS flags (graph-capturable)
            self.hit[m].logical_or_(nxt.eq(self._eos))

    # ------------------------------------------------------------------ vocab-split head
    def _vs_graphed(self, kind: str, m: int, fn):
        """Run a vocab-split step of micro-batch m (``fn(m)`` -> its output tensors or None) eagerly
        the first time, then from a HIP graph captured on the second call (a pool per lane, apart
        from the decode graphs' pools), replayed afterwards; the captured outputs are static,
        returned on every call."""
        if not self.graphs_ok:
            return fn(m)
        key = (kind, m)
        g = self._vs_graphs.get(key)
        if g is None:
            if key not in self._vs_warm:
                self._vs_warm.add(key)
                return fn(m)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            lane = m % self.L                     # one pool per lane: lanes replay concurrently
            with torch.cuda.graph(g, pool=self._vs_pools.get(lane), capture_error_mode="thread_local"):
                self._vs_outs[key] = fn(m)
            if lane not in self._vs_pools:
                self._vs_pools[lane] = g.pool()
            self._vs_graphs[key] = g
        g.replay()
        return self._vs_outs[key]

    def _vs_shard(self, m: int):
        """This rank's logits slice + sampler phase 1 for micro-batch m (rows in hfin[m])."""
        def body(m):
            c = self.shard.candidates(self.hfin[m], self.seen[m], self.sampling, self.rng[m])
            if not self.is_first:
                self.rng[m][1:].add_(1)               # rank 0 advances after its merge (same step)
            return c
        self.cand[m] = self._vs_graphed("shard", m, body)

    def _vs_seen(self, m: int):
        """Ranks >= 1: mark the token rank 0 sent for micro-batch m in this shard's penalty flags."""
        self._vs_graphed("seen", m, lambda m: ops.seen_mark(self.seen[m], self.tokin[m], self.shard.v0))

    def _vs_merge(self, m: int):
        """Rank 0: phase 2 over every shard's candidates -> the token of each row of m."""
        self._vs_graphed("merge", m, self._vs_merge_body)

    def _vs_merge_body(self, m: int):
        sp = self.sampling
        nxt = ops.sample_merge([self.cand[m]] + self.cand_in[m], self.cfg.vocab_size, sp.temperature, sp.top_k,
                               sp.top_p, self.rng[m], sp.do_sample)
        self.tok[m].copy_(nxt)
        self.out[m].scatter_(1, self.step[m].view(1, 1).expand(self.b, 1), nxt.view(self.b, 1))
        self.rng[m][1:].add_(1)
        self.step[m].add_(1)
        ops.seen_mark(self.seen[m], nxt, self.shard.v0)
        if self._eos is not None:
            self.hit[m].logical_or_(nxt.eq(self._eos))

    def _vs_seen_init(self, ids: torch.Tensor, m: int):
        """Mark prompt ids [b, T] that fall in this rank's vocab shard (pads already replaced)."""
        Vs, v0 = self.shard.Vs, self.shard.v0
        j = ids.to(self.device) - v0
        j = torch.where((j >= 0) & (j < Vs), j, torch.full_like(j, Vs))
        tmp = torch.zeros(self.b, Vs + 1, dtype=torch.uint8, device=self.device)
        tmp.scatter_(1, j, 1)
        self.seen[m].bitwise_or_(tmp[:, :Vs])

    def _bucket(self, max_len: int) -> int:
        return min(self.max_seq, ((max_len + GRAPH_BUCKET - 1) // GRAPH_BUCKET) * GRAPH_BUCKET)

    def _capture(self, m: int, bucket: int):
        g = torch.cuda.CUDAGraph()
        lane = m % self.L
        # thread-local capture so the process group's watchdog thread may keep querying its
        # events meanwhile; the caller guarantees no P2P of this rank is in flight
        with torch.cuda.graph(g, pool=self._pools.get(lane), capture_error_mode="thread_local"):
            self._decode_body(m, bucket)
        if lane not in self._pools:
            self._pools[lane] = g.pool()
        self._graphs[(m, bucket)] = g
        return g

    def _decode(self, m: int, max_len: int):
        if not self.graphs_ok:
            return self._decode_body(m, max_len)
        bucket = self._bucket(max_len)
        g = self._graphs.get((m, bucket))
        if g is None:
            if not self._warm.get(m):
                self._warm[m] = True
                return self._decode_body(m, bucket)     # first decode of m runs eagerly (warm-up)
            # capture every bucket this run will reach for m at once (capture records, it does
            # not execute), so no capture — and no device synchronize — lands later in the run
            torch.cuda.synchronize(self.device)
            b = bucket
            while True:
                if (m, b) not in self._graphs:
                    self._capture(m, b)
                if b >= self._final_bucket:
                    break
                b = self._bucket(b + 1)
            g = self._graphs[(m, bucket)]
        g.replay()

    # ------------------------------------------------------------------ schedule
    @torch.no_grad()
    def run(self, prompts: Optional[Sequence[torch.Tensor]], prompt_len: int, sampling: SamplingParams,
            decode_steps: int, seed: int = 0, hook: Optional[Callable[[int], None]] = None,
            watchdog=None, fault: Optional[Callable[[int], None]] = None,
            stats_window: Optional[Tuple[int, int]] = None, prompt_lens: Optional[torch.Tensor] = None,
            eos_token_id: Optional[int] = None, eos_every: int = 8) -> PipelineResult:
        """prompts: M tensors [b, T] of token ids (needed on rank 0 only; T = prompt_len).
        decode_steps = tokens generated per sequence after the first (prefill-sampled) one.
        ``watchdog`` (parallel.watchdog.Watchdog) gets a heartbeat per tick; ``fault(tick)`` is a
        test hook that may delay or raise before a tick's exchange (fault injection).
        ``stats_window=(t_a, t_b)``: ticks over which this rank's compute / P2P-wait / bubble
        statistics are taken (``PipelineResult.stats``).
        ``prompt_lens`` [M, b] (every rank): ragged prompts right-padded to T; the last rank then
        needs ``prompts`` too (repetition-penalty history without the pads).
        ``eos_token_id``: every ``eos_every`` decode rounds all ranks agree (one all-reduce) whether
        every sequence has produced EOS, and stop together at that tick."""
        M, P, b, T = self.M, self.world, self.b, prompt_len
        S = decode_steps
        assert T + S + 1 <= self.max_seq
        V = self.cfg.vocab_size
        self.sampling = sampling
        dev = self.device
        self._plen = None
        if prompt_lens is not None:
            pl = prompt_lens.to(dev, torch.int32).view(M, b)
            assert int(pl.max()) <= T and int(pl.min()) >= 1
            if int(pl.min()) < T:
                self._plen = [pl[m].clone() for m in range(M)]
        # vocab-split head for this run (when the sampling configuration shards); the sampling rank
        # owns the tokens: rank 0 under the split (it merges), else the last stage
        self.vs = self.vs_req and ops.shard_mode(sampling.temperature, sampling.top_k, sampling.top_p, V,
                                                 sampling.do_sample) >= 0
        samp = self.is_first if self.vs else self.is_last
        self._samp = samp
        self._eos = (torch.tensor(int(eos_token_id), dtype=torch.long, device=dev)
                     if eos_token_id is not None and samp else None)
        if samp:
            self.hit = [torch.zeros(b, dtype=torch.bool, device=dev) for _ in range(M)]
        if self.h_on is not None:
            self._build_offload_kv(T)
        self.graphs_ok = self.use_graphs and not needs_host_sampler(sampling, V) and \
            getattr(self.kv, "graph_safe", True) and \
            all(getattr(mm, "graph_safe", True) or getattr(mm, "graph_safe_rows", 0) >= b for mm in self.model.modules())
        self._warm: Dict[int, bool] = {}
        self._graphs.clear()
        self._pools.clear()
        self._vs_graphs: Dict[tuple, object] = {}
        self._vs_outs: Dict[tuple, object] = {}
        self._vs_warm = set()
        self._vs_pools: Dict[int, object] = {}
        self._final_bucket = self._bucket(T + S + 1)
        if self.vs or self.is_last:
            Vs = self.shard.Vs if self.vs else V
            self.seen = [torch.zeros(b, Vs, dtype=torch.uint8, device=dev) for _ in range(M)]
            self.rng = [torch.tensor([(seed + 7919 * m) & 0x7FFFFFFF, 0], dtype=torch.int32, device=dev)
                        for m in range(M)]
        if samp:
            self.step = [torch.zeros(1, dtype=torch.long, device=dev) for _ in range(M)]
            self.out = [torch.zeros(b, S + 1, dtype=torch.long, device=dev) for _ in range(M)]
        if self.is_last and not self.vs:
            self.ctr = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(M)]   # sampler counters
        if self.vs:
            H = self.cfg.hidden_size
            mode = ops.shard_mode(sampling.temperature, sampling.top_k, sampling.top_p, V, sampling.do_sample)
            self.hfin = [torch.zeros(b, H, dtype=self.model.dtype, device=dev) for _ in range(M)]
            self.cand: Dict[int, tuple] = {}
            if self.is_first:                        # receive buffers for the other ranks' candidates
                vb = self.vs_bounds
                self.cand_in = [[tuple(torch.empty(shp, dtype=dt, device=dev) for shp, dt in
                                       ops.shard_candidate_shapes(b, vb[r + 1] - vb[r], V, mode, dev))
                                 for r in range(1, P)] for _ in range(M)]
            else:
                self.tokin = [torch.zeros(b, dtype=torch.long, device=dev) for _ in range(M)]
        # repetition-penalty history needs the prompt ids on the sampling rank(s)
        pdev = "cpu" if self.host_staged else dev
        if self.vs:
            if self.is_first:
                stacked = torch.stack([p.to(pdev) for p in prompts])
                for r in range(1, P):
                    self._send_one(stacked, r)
            else:
                stacked = torch.zeros(M, b, T, dtype=torch.long, device=pdev)
                self._recv_one(stacked, 0)
            for m in range(M):
                ids = stacked[m].to(dev)
                if self._plen is not None:              # pads repeat the row's first token
                    pos = torch.arange(T, device=dev)[None, :]
                    ids = torch.where(pos < self._plen[m][:, None], ids, ids[:, :1])
                self._vs_seen_init(ids, m)
        elif self.is_last:
            if self.is_first or (prompts is not None and prompt_lens is not None):
                for m in range(M):
                    ids = prompts[m].to(dev)
                    if self._plen is not None:          # pads repeat the row's first token
                        pos = torch.arange(T, device=dev)[None, :]
                        ids = torch.where(pos < self._plen[m][:, None], ids, ids[:, :1])
                    self.seen[m].scatter_(1, ids, 1)
            else:
                pids = torch.zeros(M, b, T, dtype=torch.long, device=pdev)
                self._recv_one(pids, 0)
                pids = pids.to(dev)
                for m in range(M):
                    self.seen[m].scatter_(1, pids[m], 1)
        elif self.is_first and P > 1 and prompt_lens is None:
            self._send_one(torch.stack([p.to(pdev) for p in prompts]), P - 1)

        H = self.cfg.hidden_size
        pre_in = [None] * M
        pre_out = [None] * M
        n_items = M + S * M

        def feeds_back(i):  # does item i's sampled token feed a later decode item?
            return (i < M and S >= 1) or (i >= M and (i - M) // M + 1 < S)

        # tick t: rank r processes item group t - D r (items [g L, (g + 1) L), one per lane, on the
        # lanes' streams).  D = 1 + slack ticks separate a group's visits of adjacent stages.  Every
        # tick posts ONE grouped exchange: the outputs of this rank's previous tick out, the inputs
        # of the group it computes at tick t + D - 1 in (and on stage 0 the tokens the last stage
        # sampled at tick t - 1).  D = 1: the exchange completes before this tick's compute, which
        # needs it.  D = 2: it completes one tick later, so the hop runs beside a whole tick of
        # compute — at the price of 2P micro-batches in flight (the token ring then has 2P ticks).
        L = self.L
        D = 1 + self.slack
        assert D == 1 or M // L >= D * (P - 1) + 2 or P == 1, \
            f"slack {self.slack} needs >= {D * (P - 1) + 2} micro-batch groups in flight, have {M // L}"
        # vocab split: group g's hidden leaves the last stage at tick g + D(P-1), every rank runs its
        # head shard at g + DP, rank 0 merges at g + D(P+1) and feeds the token to the group's next
        # step, which starts there at g + M/L
        assert not self.vs or M // L >= D * (P + 1), \
            f"vocab split needs >= {D * (P + 1)} micro-batch groups in flight, have {M // L}"
        n_groups = n_items // L
        cur_stream = torch.cuda.current_stream(dev) if self.cuda else None
        R = D * self.rank                               # this rank's tick offset

        def group_valid(g):
            return 0 <= g < n_groups

        def lane_ctx(i):
            return torch.cuda.stream(self.streams[i % L]) if self.streams else _nullctx()

        w_a, w_b = stats_window if stats_window is not None else (-1, -1)
        ev_in: Dict[int, object] = {}      # tick -> inputs ready (exchange done)
        ev_done: Dict[int, object] = {}    # tick -> all lanes' compute done
        win_bytes = 0

        def mark(store, t):
            if self.cuda:
                e = torch.cuda.Event(enable_timing=True)
                e.record(cur_stream)
                store[t] = e
            else:
                store[t] = time.perf_counter()

        t_start = time.perf_counter()
        n_ticks = n_groups + D * (P + 1 if self.vs else P - 1)
        # EOS agreement: from the tick after which the last stage has sampled every micro-batch's
        # first token, once per eos_every decode rounds (M / L ticks per round)
        eos_on = eos_token_id is not None and (P == 1 or dist.is_initialized())
        eos_from, eos_period = (M // L) + D * (P + 1 if self.vs else P - 1), max(1, eos_every) * max(1, M // L)
        stopped_at = None
        # tick whose prefill samples the first token (vocab split: rank 0's first merge)
        t_first = (D * (P + 1) if self.is_first else -1) if self.vs else (D * (P - 1) if self.is_last else -1)
        ev_first: Dict[int, object] = {}
        mark(ev_first, -1)
        due: Dict[int, object] = {}         # tick -> posted exchange whose receives it computes on
        done_ev: Dict[int, object] = {}     # tick -> event after its compute (host-staged sends)
        host_late = self.host_staged and D > 1

        # lanes on GPU streams: every lane posts and completes its OWN exchange on its stream, so a
        # lane's hop waits only for that lane's compute and overlaps the other lanes' compute, and no
        # lane waits at a tick boundary for the others (items of different lanes never share data)
        per_lane = self.streams is not None

        def exchange_for(t, lanes):
            """(sends, recvs) of the exchange posted at tick t for the given lanes of the group."""
            prv_g, rcv_g = t - 1 - R, t + D - 1 - R
            sends, recvs = [], []
            if P == 1:
                return sends, recvs
            if group_valid(prv_g):
                for prv in (prv_g * L + l for l in lanes):
                    if not self.is_last:
                        sends.append((pre_out[prv] if prv < M else self.hout[(prv - M) % M], self.next))
                    elif self.vs:                       # final-normed rows to every other rank's head shard
                        sends.extend((self.hfin[prv % M], r) for r in range(P - 1))
                    elif feeds_back(prv):
                        sends.append((self.tok[prv % M], 0))
            if not self.is_first and group_valid(rcv_g):
                for cur in (rcv_g * L + l for l in lanes):
                    if cur < M:
                        pre_in[cur] = torch.empty(b * T, H, dtype=self.model.dtype, device=dev)
                        recvs.append((pre_in[cur], self.prev))
                    else:
                        recvs.append((self.hin[(cur - M) % M], self.prev))
            if self.is_first and not self.vs:
                prod_g = t - 1 - D * (P - 1)    # group the last stage finished at tick t - 1
                if group_valid(prod_g):
                    for prod in (prod_g * L + l for l in lanes):
                        if feeds_back(prod):
                            recvs.append((self.tok[prod % M], P - 1))
            if self.vs:                # (after the hand-offs: P2P ops of a rank pair match in posting order)
                hg, cg, mg = t - 1 - D * (P - 1), t - 1 - D * P, t - 1 - D * (P + 1)
                if not self.is_last and group_valid(hg):
                    recvs.extend((self.hfin[i % M], P - 1) for i in (hg * L + l for l in lanes))
                if group_valid(cg):
                    for i in (cg * L + l for l in lanes):
                        if self.is_first:
                            recvs.extend((x, r + 1) for r, c in enumerate(self.cand_in[i % M]) for x in c)
                        else:
                            sends.extend((x, 0) for x in self.cand[i % M])
                if group_valid(mg):
                    for i in (mg * L + l for l in lanes):
                        if feeds_back(i):
                            if self.is_first:
                                sends.extend((self.tok[i % M], r) for r in range(1, P))
                            else:
                                recvs.append((self.tokin[i % M], 0))
            return sends, recvs

        def post(t):
            nonlocal win_bytes
            parts = [(l,) for l in range(L)] if per_lane else [tuple(range(L))]
            handles = []
            for lanes in parts:
                # under the lane's stream: receive buffers are allocated on it, the sends wait on it
                with (lane_ctx(lanes[0]) if per_lane else _nullctx()):
                    sends, recvs = exchange_for(t, lanes)
                    if w_a <= t < w_b:
                        win_bytes += sum(x.numel() * x.element_size() for x, _ in sends)
                    ready = done_ev.pop((t - 1, lanes[0]), None) if host_late else None
                    handles.append(self._post(sends, recvs, send_ready=ready,
                                              group=self.lane_groups[lanes[0]] if per_lane else None))
            due[t + D - 1] = handles
            if not self.is_last:
                for prv in range((t - 1 - R) * L, (t - R) * L):
                    if 0 <= prv < M:
                        pre_out[prv] = None             # handed to the exchange (it holds the tensor)

        def finish(t):
            for i, h in enumerate(due.pop(t, None) or []):
                with (lane_ctx(i) if per_lane else _nullctx()):
                    self._finish(h)

        def mark_on(store, t):                   # per-lane mode: one event per lane stream
            if per_lane:
                store[t] = []
                for st in self.streams:
                    e = torch.cuda.Event(enable_timing=True)
                    e.record(st)
                    store[t].append(e)
            else:
                mark(store, t)

        if per_lane:
            for st in self.streams:
                st.wait_stream(cur_stream)
        # host time the loop spends per tick in the window (us): posting / completing the exchanges
        # and issuing the compute (graph replays).  With RCCL none of it blocks on the device, so it
        # is the pipeline's host overhead per tick (verdict r4: host_issue_us_per_tick)
        host_us = {"post": 0.0, "finish": 0.0, "compute": 0.0}
        pc = time.perf_counter
        for t in range(n_ticks):
            if hook is not None:
                hook(t)
            if watchdog is not None:
                watchdog.beat(f"rank {self.rank} tick {t}/{n_ticks}")
            if fault is not None:
                fault(t)
            cur_g = t - R
            in_win = w_a <= t < w_b
            if w_a <= t - 1 < w_b:
                mark_on(ev_done, t - 1)
            h0 = pc()
            if not host_late:
                post(t)                                  # before this tick's compute: the hop overlaps it
            h1 = pc()
            finish(t)
            h2 = pc()
            if in_win:
                host_us["post"] += (h1 - h0) * 1e6
                host_us["finish"] += (h2 - h1) * 1e6
            if w_a <= t < w_b:
                mark_on(ev_in, t)
            h3 = pc()
            if self.vs:                                  # head shards, rank 0's merges, penalty flags
                with trace_range(f"pp.vocab{t}"):
                    if not self.is_first and group_valid(t - D * (P + 2)):
                        for cur in range((t - D * (P + 2)) * L, (t - D * (P + 2)) * L + L):
                            if feeds_back(cur):
                                with lane_ctx(cur):
                                    self._vs_seen(cur % M)
                    if self.is_first and group_valid(t - D * (P + 1)):
                        for cur in range((t - D * (P + 1)) * L, (t - D * (P + 1)) * L + L):
                            with lane_ctx(cur):
                                self._vs_merge(cur % M)
                    if group_valid(t - D * P):
                        for cur in range((t - D * P) * L, (t - D * P) * L + L):
                            with lane_ctx(cur):
                                self._vs_shard(cur % M)
            if group_valid(cur_g):
                with trace_range(f"pp.tick{t}"):
                    for cur in range(cur_g * L, cur_g * L + L):
                        with lane_ctx(cur):
                            if cur < M:                           # prefill item
                                m = cur
                                ids = prompts[m].to(dev) if self.is_first else None
                                out = self._prefill(m, ids, T, pre_in[m])
                                pre_in[m] = None
                                if self.is_last and self.vs:
                                    self.hfin[m].copy_(out)
                                elif self.is_last:
                                    self._sample(m, out)
                                else:
                                    pre_out[m] = out
                            else:
                                k, m = divmod(cur - M, M)
                                self._decode(m, T + k + 1)
            if in_win:
                host_us["compute"] += (pc() - h3) * 1e6
            if host_late:
                # host-staged slack: this tick's compute is queued first, then the exchange whose
                # sends are the previous tick's outputs (the host waits only for that tick)
                for lanes in ([(l,) for l in range(L)] if per_lane else [tuple(range(L))]):
                    e = torch.cuda.Event()
                    e.record(self.streams[lanes[0]] if per_lane else cur_stream)
                    done_ev[(t, lanes[0])] = e
                post(t)
            debug_sync(f"pp.tick{t}")
            if t == t_first:
                if self.streams:
                    for st in self.streams:
                        cur_stream.wait_stream(st)
                mark(ev_first, t)
            if eos_on and t >= eos_from and (t - eos_from) % eos_period == 0 and t < n_ticks - 1:
                if per_lane:
                    for st in self.streams:
                        cur_stream.wait_stream(st)
                if self._all_hit():
                    stopped_at = t
                    break
        for k in sorted(due):                            # (after an EOS stop: drain posted exchanges)
            finish(k)
        if self.streams:
            for st in self.streams:
                cur_stream.wait_stream(st)
        if w_a <= n_ticks - 1 < w_b:
            mark_on(ev_done, n_ticks - 1)
        if self.cuda:
            torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t_start
        stats = {}
        if stats_window is not None and ev_in:
            stats = self._window_stats(ev_in, ev_done, w_a, w_b, win_bytes)
            nwin = max(1, min(w_b, n_ticks) - w_a)
            stats.update({f"host_{k}_us_per_tick": v / nwin for k, v in host_us.items()})
            stats["host_issue_us_per_tick"] = sum(host_us.values()) / nwin
        if t_first >= 0 and t_first in ev_first:
            a, z = ev_first[-1], ev_first[t_first]
            stats["ttft_ms"] = a.elapsed_time(z) if self.cuda else (z - a) * 1e3
        toks = None
        if samp:
            toks = []
            for m in range(M):
                toks.extend(self.out[m].tolist())
        if stopped_at is not None:
            stats["eos_stop_tick"] = stopped_at
        return PipelineResult(toks, n_ticks if stopped_at is None else stopped_at + 1, elapsed, stats=stats)

    def _all_hit(self) -> bool:
        """Every rank joins: True when the sampling rank (the last stage; rank 0 under the vocab
        split) has seen EOS in every row (one all-reduce of a device flag; the host waits for it, once
        per check period)."""
        if self._samp:
            if self.streams:
                cur = torch.cuda.current_stream(self.device)
                for st in self.streams:
                    cur.wait_stream(st)
            flag = torch.stack([h.all() for h in self.hit]).all().to(torch.int32).view(1)
        else:
            flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        if self.world > 1:
            f = flag if self.nccl else flag.cpu()
            dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
            flag = f
        return bool(flag.item())

    def _window_stats(self, ev_in, ev_done, t_a, t_b, nbytes) -> Dict[str, float]:
        """Per-tick compute (inputs ready -> all lanes done) and P2P wait (lanes done -> next
        inputs ready) on this rank, milliseconds; bubble = 1 - compute / window span."""
        ticks = [t for t in range(t_a, t_b) if t in ev_in and t in ev_done]
        if not ticks:
            return {}
        if isinstance(ev_in[ticks[0]], list):
            return self._window_stats_lanes(ev_in, ev_done, ticks, t_b - t_a, nbytes)
        if self.cuda:
            dt = lambda a, b: a.elapsed_time(b)             # noqa: E731
        else:
            dt = lambda a, b: (b - a) * 1e3                 # noqa: E731
        busy = [dt(ev_in[t], ev_done[t]) for t in ticks]
        waits = [dt(ev_done[t - 1], ev_in[t]) for t in ticks if t - 1 in ev_done]
        span = dt(ev_in[ticks[0]], ev_done[ticks[-1]])
        busy_s = sorted(busy)
        return dict(ticks=len(ticks), compute_ms_per_tick=sum(busy) / len(busy),
                    compute_ms_p50=busy_s[len(busy_s) // 2],
                    p2p_wait_ms_per_tick=(sum(waits) / len(waits)) if waits else 0.0,
                    span_ms=span, bubble_frac=max(0.0, 1.0 - sum(busy) / span) if span > 0 else 0.0,
                    p2p_bytes_per_tick=nbytes / max(1, t_b - t_a))


    @staticmethod
    def _window_stats_lanes(ev_in, ev_done, ticks, n_ticks, nbytes) -> Dict[str, float]:
        """Per-lane exchanges: a lane computes from its inputs' arrival to its own done event, and
        the lanes overlap, so the busy time is the UNION of every lane's compute intervals; the P2P
        wait is each lane's done(t - 1) -> inputs(t), averaged over lanes."""
        ref = ev_in[ticks[0]][0]
        at = lambda e: ref.elapsed_time(e)                  # noqa: E731
        iv = sorted((at(ev_in[t][l]), at(ev_done[t][l])) for t in ticks for l in range(len(ev_in[t])))
        busy, (cs, ce) = 0.0, iv[0]
        for a, z in iv[1:]:
            if a > ce:
                busy, cs, ce = busy + (ce - cs), a, z
            else:
                ce = max(ce, z)
        busy += ce - cs
        waits = [at(ev_in[t][l]) - at(ev_done[t - 1][l]) for t in ticks if t - 1 in ev_done
                 for l in range(len(ev_in[t]))]
        span = max(z for _, z in iv) - min(a for a, _ in iv)
        busy_t = [max(at(ev_done[t][l]) for l in range(len(ev_in[t]))) - min(at(ev_in[t][l]) for l in range(len(ev_in[t])))
                  for t in ticks]
        busy_s = sorted(busy_t)
        return dict(ticks=len(ticks), compute_ms_per_tick=busy / len(ticks), compute_ms_p50=busy_s[len(busy_s) // 2],
                    p2p_wait_ms_per_tick=(sum(waits) / len(waits)) if waits else 0.0, span_ms=span,
                    bubble_frac=max(0.0, 1.0 - busy / span) if span > 0 else 0.0,
                    p2p_bytes_per_tick=nbytes / max(1, n_ticks))


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def init_distributed(backend: Optional[str] = None, timeout_s: Optional[float] = None):
    """torchrun-style init (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*). backend "nccl" is RCCL.

    With RCCL the rank's GPU is bound at init (``device_id``): the world communicator is created
    eagerly, so the first grouped P2P does not build one lazily inside the decode loop.
    ``timeout_s`` (default ``EDGELLM_PG_TIMEOUT_S`` or 600) bounds every collective / P2P wait."""
    import os
    from .watchdog import init_pg_timeout
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    backend = os.environ.get("EDGELLM_DIST_BACKEND", backend)   # e.g. gloo: GPU ranks sharing one device
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    timeout = init_pg_timeout(float(os.environ.get("EDGELLM_PG_TIMEOUT_S", timeout_s or 600.0)))
    kw = {}
    if backend == "nccl":
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
        kw["device_id"] = dev
    dist.init_process_group(backend=backend, timeout=timeout, **kw)
    return dist.get_rank(), dist.get_world_size()
