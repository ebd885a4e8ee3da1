"""Layer-partitioned inference pipeline: one process per GPU ("edge device"), RCCL P2P over xGMI.

The reference only ever splits a model implicitly through accelerate's ``device_map="auto"``
(activations hop GPUs via ``tensor.to(next_device)``, no micro-batching — SURVEY §2.4, K16) and
ships no tensors over its gRPC demo.  Here every stage is its own process; hidden states move
rank r -> r+1 with RCCL point-to-point, and the tokens sampled on the last stage travel back to
stage 0 (a token ring), so decode keeps every stage busy:

  work items (same order on every rank):  prefill(m) for m < M, then decode(k, m) for k < S
  rank s processes item i at tick i + s (lockstep); with M >= P micro-batches the token of
  decode(k, m) reaches stage 0 exactly when decode(k+1, m) starts (M - P ticks of slack).

Per tick each rank issues ONE grouped P2P exchange (send the previous tick's output, receive
this tick's input — grouped, so no send/recv ordering deadlock), then runs its layers for the
micro-batch.  The decode compute of each micro-batch is captured in a HIP graph (per KV-length
bucket); the P2P ops stay outside the graph on RCCL's stream, ordered by stream waits, so the
host never blocks on the device inside the loop.  Messages: decode b*H*2 bytes per hop
(16 x 4096 bf16 = 128 KiB), prefill b*T*H*2.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import ops
from ..engine.generate import GRAPH_BUCKET, SamplingParams, needs_host_sampler
from ..engine.kv_cache import KVCache
from ..models.decoder import AttnCtx, DecoderLM


@dataclass
class PipelineResult:
    tokens: Optional[List[List[int]]]    # last rank: generated ids per sequence (micro-batch major)
    ticks: int
    elapsed_s: float
    marks: Dict[str, float] = field(default_factory=dict)


class PipelineStage:
    def __init__(self, model: DecoderLM, rank: int, world: int, micro_batch: int, n_micro: int, max_seq: int,
                 group=None, use_graphs: Optional[bool] = None, headinfer_heads: Optional[int] = None,
                 lanes: int = 1):
        """``headinfer_heads``: keep only this many KV heads per layer on the GPU and offload the rest
        to pinned host memory (edgellm.offload.HeadInferKV; BASELINE config "8-way pipeline +
        HeadInfer").  The offloaded path is host-orchestrated, so its decode steps run eagerly."""
        assert lanes >= 1 and n_micro % lanes == 0, "micro-batches must split evenly over lanes"
        assert n_micro >= world * lanes, "need lanes x stages micro-batches to keep the ring full"
        self.model, self.cfg = model, model.cfg
        self.rank, self.world = rank, world
        self.b, self.M = micro_batch, n_micro
        self.max_seq = max_seq
        self.group = group
        self.device = model.device
        self.first, self.last = model.first, model.last
        self.is_first, self.is_last = model.has_embed, model.has_head
        assert self.is_first == (rank == 0) and self.is_last == (rank == world - 1)
        self.prev = (rank - 1) % world
        self.next = (rank + 1) % world
        if headinfer_heads is not None and headinfer_heads < self.cfg.num_kv_heads:
            from ..offload import HeadInferKV
            self.kv = HeadInferKV(self.cfg, micro_batch * n_micro, max_seq, headinfer_heads, self.device, self.first,
                                  self.last, chunk_size=max_seq, dtype=model.dtype)
        else:
            self.kv = KVCache(self.cfg, micro_batch * n_micro, max_seq, self.first, self.last, model.dtype,
                              self.device)
        self.attn_hook = getattr(self.kv, "attn_hook", None)
        self.rope = model.rope_table(self.device)
        cuda = self.device.type == "cuda"
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

    # ------------------------------------------------------------------ p2p
    def _exchange(self, sends, recvs):
        """sends/recvs: lists of (tensor, peer).  One grouped exchange."""
        if not sends and not recvs:
            return
        if self.nccl:
            p2p = [dist.P2POp(dist.isend, t, p, self.group) for t, p in sends]
            p2p += [dist.P2POp(dist.irecv, t, p, self.group) for t, p in recvs]
            for w in dist.batch_isend_irecv(p2p):
                w.wait()
        elif self.host_staged:
            works = [dist.isend(t.cpu(), p, self.group) for t, p in sends]
            bufs = [torch.empty(t.shape, dtype=t.dtype) for t, _ in recvs]
            works += [dist.irecv(h, p, self.group) for h, (_, p) in zip(bufs, recvs)]
            for w in works:
                w.wait()
            for h, (t, _) in zip(bufs, recvs):
                t.copy_(h)
        else:
            works = [dist.isend(t, p, self.group) for t, p in sends]
            works += [dist.irecv(t, p, self.group) for t, p in recvs]
            for w in works:
                w.wait()

    # ------------------------------------------------------------------ compute
    def _rows(self, m):
        return self.kv.rows(m * self.b, (m + 1) * self.b)

    def _prefill(self, m: int, ids: Optional[torch.Tensor], T: int, hidden: Optional[torch.Tensor]):
        b = self.b
        sp = torch.zeros(b, dtype=torch.int32, device=self.device)
        ctx = AttnCtx("prefill", b, T, sp, sp + T, T, self._rows(m), self.rope, attn_hook=self.attn_hook)
        out = self.model(ids, ctx, hidden=hidden, logits="last")
        self.pos[m].fill_(T)
        self.lens[m].fill_(T + 1)
        return out

    def _decode_body(self, m: int, max_len: int):
        b = self.b
        ctx = AttnCtx("decode", b, 1, self.pos[m], self.lens[m], max_len, self._rows(m), self.rope,
                      attn_hook=self.attn_hook)
        out = self.model(self.tok[m].view(b, 1) if self.is_first else None, ctx,
                         hidden=None if self.is_first else self.hin[m])
        if self.is_last:
            self._sample(m, out)
        else:
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

    def _decode(self, m: int, max_len: int):
        if not self.graphs_ok:
            return self._decode_body(m, max_len)
        bucket = min(self.max_seq, ((max_len + GRAPH_BUCKET - 1) // GRAPH_BUCKET) * GRAPH_BUCKET)
        key = (m, bucket)
        g = self._graphs.get(key)
        if g is None:
            if not self._warm.get(m):
                self._warm[m] = True
                return self._decode_body(m, bucket)     # first decode of m runs eagerly (warm-up)
            g = torch.cuda.CUDAGraph()
            # no P2P in flight during capture, and a thread-local capture so the process group's
            # watchdog thread may keep querying its events meanwhile
            torch.cuda.synchronize()
            lane = m % self.L
            with torch.cuda.graph(g, pool=self._pools.get(lane), capture_error_mode="thread_local"):
                self._decode_body(m, bucket)
            if lane not in self._pools:
                self._pools[lane] = g.pool()
            self._graphs[key] = g
            return g.replay()
        g.replay()

    # ------------------------------------------------------------------ schedule
    @torch.no_grad()
    def run(self, prompts: Optional[Sequence[torch.Tensor]], prompt_len: int, sampling: SamplingParams,
            decode_steps: int, seed: int = 0, hook: Optional[Callable[[int], None]] = None,
            watchdog=None, fault: Optional[Callable[[int], None]] = None) -> PipelineResult:
        """prompts: M tensors [b, T] of token ids (needed on rank 0 only; T = prompt_len).
        decode_steps = tokens generated per sequence after the first (prefill-sampled) one.
        ``watchdog`` (parallel.watchdog.Watchdog) gets a heartbeat per tick; ``fault(tick)`` is a
        test hook that may delay or raise before a tick's exchange (fault injection)."""
        M, P, b, T = self.M, self.world, self.b, prompt_len
        S = decode_steps
        assert T + S + 1 <= self.max_seq
        V = self.cfg.vocab_size
        self.sampling = sampling
        self.graphs_ok = self.use_graphs and not needs_host_sampler(sampling, V) and \
            getattr(self.kv, "graph_safe", True) and \
            all(getattr(mm, "graph_safe", True) or getattr(mm, "graph_safe_rows", 0) >= b for mm in self.model.modules())
        self._warm: Dict[int, bool] = {}
        self._graphs.clear()
        self._pools.clear()
        dev = self.device
        if self.is_last:
            self.seen = [torch.zeros(b, V, dtype=torch.uint8, device=dev) for _ in range(M)]
            self.rng = [torch.tensor([(seed + 7919 * m) & 0x7FFFFFFF, 0], dtype=torch.int32, device=dev)
                        for m in range(M)]
            self.step = [torch.zeros(1, dtype=torch.long, device=dev) for _ in range(M)]
            self.out = [torch.zeros(b, S + 1, dtype=torch.long, device=dev) for _ in range(M)]
        if self.is_first and self.is_last is False:
            pass
        # repetition-penalty history needs the prompt ids on the last stage
        if self.is_last:
            if self.is_first:
                for m in range(M):
                    self.seen[m].scatter_(1, prompts[m].to(dev), 1)
            else:
                pids = torch.zeros(M, b, T, dtype=torch.long, device="cpu" if self.host_staged else dev)
                if dist.is_initialized():
                    dist.recv(pids, 0, self.group)
                pids = pids.to(dev)
                for m in range(M):
                    self.seen[m].scatter_(1, pids[m], 1)
        elif self.is_first and P > 1:
            dist.send(torch.stack([p.to("cpu" if self.host_staged else dev) for p in prompts]), P - 1, self.group)

        H = self.cfg.hidden_size
        pre_in = [None] * M
        pre_out = [None] * M
        n_items = M + S * M

        def valid(i):
            return 0 <= i < n_items

        def feeds_back(i):  # does item i's sampled token feed a later decode item?
            return (i < M and S >= 1) or (i >= M and (i - M) // M + 1 < S)

        # tick t: rank r processes item group t - r (items [g L, (g + 1) L), one per lane, on the
        # lanes' streams); every tick starts with ONE grouped exchange (the previous group's outputs
        # out, this group's inputs in) ordered after all lanes' work and before any of the next
        L = self.L
        n_groups = n_items // L
        cur_stream = torch.cuda.current_stream(dev) if self.streams else None

        def group_valid(g):
            return 0 <= g < n_groups

        def lane_ctx(i):
            return torch.cuda.stream(self.streams[i % L]) if self.streams else _nullctx()

        t_start = time.perf_counter()
        n_ticks = n_groups + P - 1
        for t in range(n_ticks):
            if hook is not None:
                hook(t)
            if watchdog is not None:
                watchdog.beat(f"rank {self.rank} tick {t}/{n_ticks}")
            if fault is not None:
                fault(t)
            cur_g, prv_g = t - self.rank, t - 1 - self.rank
            sends, recvs = [], []
            if P > 1:
                if group_valid(prv_g):
                    for prv in range(prv_g * L, prv_g * L + L):
                        if not self.is_last:
                            sends.append((pre_out[prv] if prv < M else self.hout[(prv - M) % M], self.next))
                        elif feeds_back(prv):
                            sends.append((self.tok[prv % M], 0))
                if not self.is_first and group_valid(cur_g):
                    for cur in range(cur_g * L, cur_g * L + L):
                        if cur < M:
                            pre_in[cur] = torch.empty(b * T, H, dtype=self.model.dtype, device=dev)
                            recvs.append((pre_in[cur], self.prev))
                        else:
                            recvs.append((self.hin[(cur - M) % M], self.prev))
                if self.is_first:
                    prod_g = t - P        # group the last stage finished at tick t-1
                    if group_valid(prod_g):
                        for prod in range(prod_g * L, prod_g * L + L):
                            if feeds_back(prod):
                                recvs.append((self.tok[prod % M], P - 1))
            if self.streams:
                for st in self.streams:
                    cur_stream.wait_stream(st)
            self._exchange(sends, recvs)
            if self.streams:
                for st in self.streams:
                    st.wait_stream(cur_stream)
            if not group_valid(cur_g):
                continue
            for cur in range(cur_g * L, cur_g * L + L):
                with lane_ctx(cur):
                    if cur < M:                           # prefill item
                        m = cur
                        if self.streams and pre_in[m] is not None:
                            pre_in[m].record_stream(self.streams[m % L])   # received on the exchange stream
                        ids = prompts[m].to(dev) if self.is_first else None
                        out = self._prefill(m, ids, T, pre_in[m])
                        pre_in[m] = None
                        if self.is_last:
                            self._sample(m, out)
                        else:
                            pre_out[m] = out
                    else:
                        k, m = divmod(cur - M, M)
                        self._decode(m, T + k + 1)
            if not self.is_last and group_valid(prv_g):
                for prv in range(prv_g * L, prv_g * L + L):
                    if prv < M:
                        pre_out[prv] = None                # sent this tick
        if self.streams:
            for st in self.streams:
                cur_stream.wait_stream(st)
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - t_start
        toks = None
        if self.is_last:
            toks = []
            for m in range(M):
                toks.extend(self.out[m].tolist())
        return PipelineResult(toks, n_ticks, elapsed)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def init_distributed(backend: Optional[str] = None):
    """torchrun-style init (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*). backend "nccl" is RCCL."""
    import os
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    backend = os.environ.get("EDGELLM_DIST_BACKEND", backend)   # e.g. gloo: GPU ranks sharing one device
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()
