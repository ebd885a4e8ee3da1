"""Pipeline-parallel serving engine: the micro-batched RCCL ``PipelineStage`` behind the
``Generator`` interface, so the CLIs (evaluate / combine / serve) run a model split over
``pp_size`` GPUs as one process per GPU instead of the eager in-process ``SplitLM``.

The reference's only multi-device mechanism is accelerate's ``device_map="auto"`` layer split,
which hops the hidden state GPU to GPU with no micro-batching
(Code/Base Models/combine_model_fp_updated.py:40, Llama_bf16_updated.py:31).  Here, under
``torchrun --nproc-per-node P``:

* every rank holds stage ``rank`` of every agent's model (``load_stage``: bit-identical weights
  to the unsplit model for a layer, SmoothQuant calibrated on the full model once);
* rank 0 is the DRIVER: it runs the evaluation loop, and each ``generate`` / ``confidence``
  call broadcasts one command (a small int64 header + float sampling parameters + the padded
  prompt ids and lengths) to all ranks;
* every other rank is a WORKER in ``serve_workers``: it executes the same commands on its stage
  until the driver sends STOP;
* a command runs ``PipelineStage.run`` on every rank (ragged prompts right-padded, one prefill
  pass per micro-batch, EOS agreement every few decode rounds) and the last stage returns the
  tokens (and timings) to the driver with one P2P message.

Prompts are spread over the stage's M micro-batches of b rows; unused rows repeat prompt 0 and
are discarded.  Works on gloo (CPU, tests) and on RCCL (one GPU per rank).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import ops
from ..engine.generate import GenerationResult, SamplingParams
from ..utils.log import get_logger
from ..models.decoder import AttnCtx, DecoderLM
from .pipeline import PipelineStage
from .pp_slots import CMD_SLOT_ADMIT, CMD_SLOT_OPEN, CMD_SLOT_STEP, handle_slot_command

CMD_GENERATE, CMD_SCORE, CMD_STOP = 1, 2, 3
log = get_logger("pp_engine")
_HDR = 12


def distributed_world() -> int:
    """WORLD_SIZE of a torchrun launch (1 when not launched by torchrun)."""
    return int(os.environ.get("WORLD_SIZE", "1"))


def stage_unit_bounds(cfg, world: int, partition: str = "balanced", quant: str = "none", rows: int = 1,
                      ctx: int = 256, kv_bytes: float = 2.0) -> List[int]:
    """Stage boundaries in half-layer units (unit 2 i = layer i's attention half, 2 i + 1 its MLP
    half).  ``units``: the decode cost model (parallel.partition.partition_units) at ``rows`` rows
    and ``ctx`` cached tokens — a boundary may fall inside a layer; ``balanced`` / ``uniform`` /
    explicit "8,8,8,8": whole layers (bytes per decode step)."""
    from .partition import partition_model, partition_units
    wb = 1.0 if quant not in (None, "none") else 2.0
    if partition == "units":
        return list(partition_units(cfg, world, rows=max(1, rows), ctx=ctx, weight_bytes=wb, kv_bytes=kv_bytes))
    explicit = partition if "," in partition else None
    mode = "uniform" if partition == "uniform" else "balanced"
    return [2 * x for x in partition_model(cfg, world, mode, weight_bytes=wb, explicit=explicit)]


def _peak_build_mb(device) -> float:
    """Peak memory of this rank so far: device allocator peak on a GPU, max RSS on the CPU."""
    dev = torch.device(device)
    if dev.type == "cuda":
        return torch.cuda.max_memory_allocated(dev) / 2 ** 20
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0


def load_stage(model_id: str, precision: str, quant: str, device, base_dir: Optional[str], rank: int, world: int,
               bounds: Optional[Sequence[int]] = None, partition: str = "balanced", group=None,
               ranks: Optional[Sequence[int]] = None, calib: str = "stage", rows: int = 1, ctx: int = 256):
    """This rank's pipeline stage of ``model_id``: half-layer units [ub[rank], ub[rank+1]) of
    ``stage_unit_bounds`` (``partition``; ``bounds`` = explicit LAYER bounds), the embedding on
    stage 0, the head on the last.  Random-init weights are seeded by global parameter name, so a
    stage's weights equal the unsplit model's.

    SmoothQuant (``quant="w8a8_smoothquant"``, no int8 checkpoint):
      * ``calib="stage"`` (default under a multi-rank launch): the rank builds ONLY its stage and
        calibrates it on the activations the previous stage sends it over the pipeline's P2P
        path (``quant.smoothquant.smoothquant_stage_p2p``; every member of the group joins, in
        stage order) — no rank materialises layers it does not own;
      * ``calib="full"``: every rank builds + calibrates the full model and cuts its stage.
    An int8 checkpoint directory is read stage-locally (no calibration).
    ``group`` / ``ranks``: the model's process group and its global ranks (stage i = ranks[i]).
    Returns (stage, tokenizer, source, layer bounds; halves as .5)."""
    from ..models.registry import load_model, quantized_checkpoint_dir
    qdir = quantized_checkpoint_dir(model_id, base_dir)
    cfg, tok, source = _cfg_of(model_id, precision, torch.device("cpu"), base_dir)
    if qdir is not None:
        quant = "w8a8"          # (bytes per weight for the partition's cost model)
    if bounds is not None:
        ub = [int(round(2 * float(x))) for x in bounds]
    else:
        ub = stage_unit_bounds(cfg, world, partition, quant, rows, ctx)
    ua, ubb = ub[rank], ub[rank + 1]
    whole = ua % 2 == 0 and ubb % 2 == 0
    loc = dict(first=ua // 2, last=ubb // 2) if whole else dict(units=(ua, ubb))
    lb = [u / 2 if u % 2 else u // 2 for u in ub]
    if qdir is not None:
        # an int8 checkpoint: this rank reads only its stage (no full bf16 model, no calibration)
        stage, tok, source = load_model(qdir, precision, "none", device, None, **loc)
    elif quant == "w8a8_smoothquant":
        text = ("Question: when did the first world war begin and which countries fought in it? Answer: "
                "The First World War began in 1914 after the assassination of Archduke Franz Ferdinand.")
        ids = tok.encode(text)[:64]
        calib_ids = torch.tensor([[i % cfg.vocab_size for i in ids]], device=device)
        if calib == "stage" and world > 1 and dist.is_initialized():
            from ..quant.smoothquant import smoothquant_stage_p2p
            granks = list(ranks) if ranks is not None else list(range(world))
            nccl = dist.get_backend(group) == "nccl"
            cdev = torch.device(device) if nccl else torch.device("cpu")

            def recv_prev(shape, dtype):
                t = torch.empty(shape, dtype=dtype, device=cdev)
                dist.recv(t, granks[rank - 1], group=group)
                return t

            def send_next(t):
                dist.send(t.to(cdev).contiguous(), granks[rank + 1], group=group)

            stage = smoothquant_stage_p2p(
                cfg, calib_ids, recv_prev, send_next,
                build=lambda: load_model(model_id, precision, "none", device, base_dir, **loc)[0])
        else:
            from ..quant.smoothquant import smoothquant_stage
            full, tok, source = load_model(model_id, precision, "none", device, base_dir)
            stage = smoothquant_stage(full, loc.get("first", ua // 2), loc.get("last", ubb // 2), calib_ids,
                                      device=device, units=loc.get("units"))
            del full
    else:
        stage, tok, source = load_model(model_id, precision, quant, device, base_dir, **loc)
    nparam = sum(p.numel() * p.element_size() for p in stage.parameters()) + \
        sum(b.numel() * b.element_size() for b in stage.buffers())
    log.info(f"stage {rank}/{world} of {source}: units [{ua}, {ubb}) = layers [{lb[rank]}, {lb[rank + 1]}), "
             f"weights {nparam / 2 ** 20:.1f} MiB, peak build memory {_peak_build_mb(device):.1f} MiB "
             f"({'per-stage' if quant == 'w8a8_smoothquant' and calib == 'stage' and world > 1 else 'no'} calibration)")
    return stage, tok, source, lb


def _cfg_of(model_id, precision, device, base_dir):
    """Config + tokenizer of a model without materialising its layers (an embedding-only stage)."""
    from ..models.registry import load_model, quantized_checkpoint_dir
    qdir = quantized_checkpoint_dir(model_id, base_dir)
    if qdir is not None:
        from ..quant.checkpoint import checkpoint_config
        from ..utils.tokenizer import load_tokenizer
        cfg = checkpoint_config(qdir)
        return cfg, load_tokenizer(qdir, cfg.vocab_size), f"int8-checkpoint:{qdir}"
    from ..models.hf import resolve_model_dir
    path = resolve_model_dir(model_id, base_dir)
    if path is not None:
        # an HF checkpoint: config.json + tokenizer only (no V x H embedding read on every rank)
        from ..models.configs import from_hf_dir
        from ..utils.tokenizer import load_tokenizer
        cfg = from_hf_dir(path)
        return cfg, load_tokenizer(path, cfg.vocab_size), f"checkpoint:{path}"
    m, tok, source = load_model(model_id, precision, "none", device, base_dir, first=0, last=0)
    return m.cfg, tok, source


class _Scorer:
    """What MetricSuite's confidence metric needs from a scoring model (``confidence``)."""

    def __init__(self, engine: "PipelineGenerator"):
        self.engine = engine

    @property
    def device(self):
        return self.engine.device

    def confidence(self, ids: List[int]) -> float:
        return self.engine.confidence(ids)


class PipelineGenerator:
    """Generator-compatible front end of one model's pipeline stage on this rank.

    ``rank`` / ``world``: this rank's stage index and the stage count of the model's rank group;
    ``ranks``: the group's global ranks (default 0..world-1) and ``group`` its process group.  A
    rank outside the group holds a STUB (``stage_model=None``, ``cfg`` and ``device`` given): it
    joins the command broadcasts and skips the work, so every rank can hold one engine per agent
    and agents on disjoint rank groups decode at the same time (``generate_concurrent``).
    Commands always travel over the WORLD group from global rank 0 (the driver); results come back
    from the group's last stage to rank 0."""

    def __init__(self, stage_model: Optional[DecoderLM], rank: int, world: int, max_batch: int = 1,
                 max_seq: int = 2048, tag: int = 0, lanes: int = 1, n_micro: Optional[int] = None,
                 kv_dtype: str = "bf16", eos_every: int = 8, group=None, use_graphs: Optional[bool] = None,
                 ranks: Optional[Sequence[int]] = None, cfg=None, device=None, slack: int = 0,
                 vocab_split: bool = False, head_shard=None):
        self.rank, self.world, self.tag, self.group = rank, world, tag, group
        self.ranks = list(ranks) if ranks is not None else list(range(world))
        assert len(self.ranks) == world
        self.grank = dist.get_rank() if dist.is_initialized() else 0
        self.member = stage_model is not None
        # LM head split by vocabulary over the group (parallel/vocab_head.py): members pass their shard
        self.vs_req = bool(vocab_split) and world > 1
        M, b = self.geometry(world, max_batch, lanes, slack, n_micro, self.vs_req)
        self.M, self.b = M, b
        self.lanes, self.slack = lanes, slack
        self.cfg = stage_model.cfg if self.member else cfg
        assert self.cfg is not None, "a stub engine needs the model config"
        self.max_seq = min(max_seq, self.cfg.max_position_embeddings)   # as Generator
        if self.member:
            self.stage = PipelineStage(stage_model, rank, world, b, M, self.max_seq, group=group, lanes=lanes,
                                       kv_dtype=kv_dtype, use_graphs=use_graphs, ranks=self.ranks, slack=slack,
                                       vocab_split=self.vs_req, head_shard=head_shard)
            self.device = stage_model.device
            self.nccl = self.stage.nccl
        else:
            self.stage = None
            self.device = torch.device(device) if device is not None else torch.device("cpu")
            self.nccl = dist.is_initialized() and dist.get_backend() == "nccl"
        self.eos_every = eos_every
        self.cdev = self.device if self.nccl else torch.device("cpu")
        self.model = _Scorer(self)          # Agent / MetricSuite read generator.model
        self.last_rank = world - 1
        self.last_ticks = 0
        self.attn_hook = None               # resident KV rows: continuous batching applies (pp_slots)
        self._slot_sess = None
        self._stopped = False

    @staticmethod
    def geometry(world: int, max_batch: int, lanes: int = 1, slack: int = 0, n_micro: Optional[int] = None,
                 vocab_split: bool = False):
        """(M micro-batches, b rows each) for ``max_batch`` sequences: M covers the micro-batch
        groups a stage hop keeps in flight (P, or (1 + slack)(P - 1) + 2 with slack; (1 + slack)(P + 1)
        with the vocab-split head) times the lanes."""
        if vocab_split and world > 1:
            groups = (1 + slack) * (world + 1)
        else:
            groups = world if slack == 0 or world == 1 else (1 + slack) * (world - 1) + 2
        M = max(n_micro or 0, groups * max(1, lanes))
        M = -(-M // max(1, lanes)) * max(1, lanes)
        return M, max(1, math.ceil(max_batch / M))

    # a failure after a command went out leaves the other ranks part-way through its P2P: the
    # serving front end must not go on to the next command (serve.server.ServingEngine exits)
    fatal_on_error = True

    def slot_decoder(self, sampling: SamplingParams, seed: int = 0, width: int = 2048,
                     max_batch: Optional[int] = None):
        """Continuous-batching session over the pipeline's rows (parallel.pp_slots)."""
        from .pp_slots import PipelineSlotDecoder
        return PipelineSlotDecoder(self, sampling, seed=seed, width=width, max_batch=max_batch)

    def shutdown(self) -> None:
        """Driver: release the workers' command loop (once; ``stop_workers`` is idempotent)."""
        stop_workers(self)

    # ------------------------------------------------------------------ comm helpers
    def _bcast(self, t: torch.Tensor) -> torch.Tensor:
        """Driver -> every rank of the WORLD (command traffic)."""
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.broadcast(t, 0)
        return t

    def _result_stage(self, hdr, fl) -> int:
        """Stage whose run holds a job's tokens: 0 under the vocab split (it merges the samples)
        when the job's sampling shards, else the last; every rank derives it from the command."""
        if self.vs_req and ops.shard_mode(float(fl[0]), int(hdr[7]), float(fl[1]), self.cfg.vocab_size,
                                          bool(int(hdr[6]))) >= 0:
            return 0
        return self.world - 1

    def _deliver(self, ts: Sequence[torch.Tensor], stage: Optional[int] = None) -> None:
        """The group's result stage (default its last) -> global rank 0 (world P2P), in place on
        rank 0's buffers."""
        src = self.ranks[self.world - 1 if stage is None else stage]
        if src == 0:
            return
        for t in ts:
            if self.grank == src:
                dist.send(t, 0)
            elif self.grank == 0:
                dist.recv(t, src)

    # ------------------------------------------------------------------ driver API
    @torch.no_grad()
    def generate(self, prompts: Sequence[Sequence[int]], sampling: SamplingParams, seed: int = 0,
                 eos_token_id: Optional[int] = None, stop_at_eos: bool = True,
                 record_step_latency: bool = False) -> GenerationResult:
        return generate_concurrent([(self, prompts, sampling, seed, eos_token_id)], stop_at_eos)[0]

    @torch.no_grad()
    def confidence(self, ids: List[int]) -> float:
        """mean over positions of max softmax(logits): one pipelined prefill of ``ids`` (K13)."""
        assert self.grank == 0, "the driver (rank 0) issues commands"
        if not ids:
            return 0.0
        hdr = torch.zeros(_HDR, dtype=torch.long, device=self.cdev)
        hdr[0], hdr[1], hdr[2] = CMD_SCORE, self.tag, len(ids)
        self._bcast(hdr)
        t = self._bcast(torch.tensor(ids, dtype=torch.long, device=self.cdev))
        return self._run_score(t)

    # ------------------------------------------------------------------ every rank
    def _job_tensors(self, prompts, sampling: SamplingParams, seed: int, eos_token_id, stop_at_eos: bool):
        """Driver: the broadcast form of one generate job (header, floats, padded ids, lengths)."""
        n = len(prompts)
        assert 0 < n <= self.M * self.b, f"{n} prompts > {self.M} micro-batches x {self.b} rows"
        T = max(len(p) for p in prompts)
        assert min(len(p) for p in prompts) >= 1, "empty prompt"
        assert T + sampling.max_new_tokens <= self.max_seq, "prompt + max_new_tokens exceeds max_seq"
        rows = list(prompts) + [prompts[0]] * (self.M * self.b - n)
        ids = torch.zeros(len(rows), T, dtype=torch.long, device=self.cdev)
        for i, p in enumerate(rows):
            ids[i, :len(p)] = torch.tensor(p, dtype=torch.long)
        lens = torch.tensor([len(p) for p in rows], dtype=torch.long, device=self.cdev)
        hdr = torch.tensor([self.tag, n, T, sampling.max_new_tokens, seed,
                            -1 if eos_token_id is None or not stop_at_eos else int(eos_token_id),
                            int(sampling.do_sample), int(sampling.top_k or 0), 0, 0, 0, 0],
                           dtype=torch.long, device=self.cdev)
        fl = torch.tensor([sampling.temperature, sampling.top_p if sampling.top_p is not None else 1.0,
                           sampling.repetition_penalty, 0.0], dtype=torch.float64, device=self.cdev)
        return hdr, fl, ids, lens

    def _run_local(self, hdr, fl, ids, lens):
        """Member ranks: run the pipeline for one job; the last stage returns (tokens, timing)
        buffers, the other ranks zeros of the same shape (filled on rank 0 by ``_deliver``)."""
        n, T, max_new, seed, eos = (int(hdr[i]) for i in (1, 2, 3, 4, 5))
        out = torch.zeros(self.M * self.b, max_new, dtype=torch.long, device=self.cdev)
        timing = torch.zeros(3, dtype=torch.float64, device=self.cdev)
        if not self.member:
            return out, timing
        st = self.stage
        sp = SamplingParams(max_new_tokens=max_new, temperature=float(fl[0]), top_k=int(hdr[7]),
                            top_p=float(fl[1]), repetition_penalty=float(fl[2]), do_sample=bool(int(hdr[6])))
        M, b = st.M, st.b
        ids_d = ids.to(self.device)
        prompts = [ids_d[m * b:(m + 1) * b] for m in range(M)]
        res = st.run(prompts, T, sp, max_new - 1, seed=seed, prompt_lens=lens.view(M, b),
                     eos_token_id=None if eos < 0 else eos, eos_every=self.eos_every)
        if res.tokens is not None:                   # the sampling stage (last, or 0 under the vocab split)
            out.copy_(torch.tensor(res.tokens, dtype=torch.long))
            timing[0] = res.elapsed_s
            timing[1] = res.stats.get("ttft_ms", 0.0) / 1e3
            timing[2] = res.ticks
        return out, timing

    def _run_score(self, ids: torch.Tensor) -> float:
        """One prefill of [1, T] through the stages (micro-batch 0's cache row 0); the value
        reaches rank 0 from the last stage."""
        val = torch.zeros(1, dtype=torch.float64, device=self.cdev)
        if self.member:
            st, dev = self.stage, self.device
            T = ids.numel()
            assert T <= self.max_seq
            H = self.cfg.hidden_size
            sp = torch.zeros(1, dtype=torch.int32, device=dev)
            ctx = AttnCtx("prefill", 1, T, sp, sp + T, T, st.kv.rows(0, 1), st.rope)
            hidden = None
            if not st.is_first:
                hidden = torch.empty(T, H, dtype=st.model.dtype, device=dev if self.nccl else "cpu")
                dist.recv(hidden, st.granks[st.prev], group=self.group)
                hidden = hidden.to(dev)
            out = st.model(ids.to(dev).view(1, T) if st.is_first else None, ctx, hidden=hidden, logits="all")
            if st.is_last:
                val[0] = float(ops.max_softmax_prob(out).mean())
            else:
                dist.send(out.contiguous() if self.nccl else out.contiguous().cpu(), st.granks[st.next],
                          group=self.group)
        self._deliver([val])
        return float(val[0])


def generate_concurrent(jobs: Sequence[tuple], stop_at_eos: bool = True) -> List[GenerationResult]:
    """Driver (rank 0): run several pipeline engines' generate jobs with ONE command —
    ``jobs`` = [(engine, prompts, sampling, seed, eos_token_id)].  Every rank runs the jobs of
    the groups it belongs to in job order, so engines on DISJOINT rank groups decode at the same
    time (the reference runs its agents one after another: combine_model_fp_updated.py:194-200);
    overlapping groups run one after another in that order.  Results then travel last stage ->
    rank 0 in job order (after all compute, so no send waits on a rank still computing)."""
    eng0 = jobs[0][0]
    assert eng0.grank == 0, "the driver (rank 0) issues commands; workers run serve_workers()"
    # every job is validated and packed BEFORE the command goes out: a job rejected after the
    # header was broadcast would leave the workers blocked in the next broadcast
    packed = [(eng, *eng._job_tensors(prompts, sp, seed, eos, stop_at_eos)) for eng, prompts, sp, seed, eos in jobs]
    cmd = torch.zeros(_HDR, dtype=torch.long, device=eng0.cdev)
    cmd[0], cmd[1] = CMD_GENERATE, len(jobs)
    eng0._bcast(cmd)
    payload = []
    for eng, hdr, fl, ids, lens in packed:
        for t in (hdr, fl, ids, lens):
            eng._bcast(t)
        payload.append((eng, hdr, fl, ids, lens))
    outs = _run_jobs(payload)
    results = []
    for (eng, prompts, sp, _, eos), (out, timing) in zip(jobs, outs):
        toks = out.tolist()[:len(prompts)]
        eng.last_ticks = int(timing[2])              # ticks run (fewer when EOS ended the run)
        done = []
        for r in toks:
            if eos is not None and stop_at_eos and eos in r:
                r = r[:r.index(eos) + 1]
            done.append(r)
        elapsed, ttft = float(timing[0]), float(timing[1])
        results.append(GenerationResult(done, [len(p) for p in prompts], elapsed, ttft, max(0.0, elapsed - ttft)))
    return results


def _run_jobs(payload):
    """Every rank: compute its member jobs in order, then deliver each job's result to rank 0."""
    outs = [eng._run_local(hdr, fl, ids, lens) for eng, hdr, fl, ids, lens in payload]
    for (eng, hdr, fl, *_), o in zip(payload, outs):
        eng._deliver(list(o), eng._result_stage(hdr, fl))
    return outs


def serve_workers(engines: Dict[int, PipelineGenerator]) -> int:
    """Worker loop of ranks > 0: execute the driver's commands on the stages this rank holds
    (every agent has an engine here, a stub where the rank is outside the agent's group) until
    STOP.  Returns the number of commands served."""
    any_eng = next(iter(engines.values()))
    served = 0
    while True:
        hdr0 = any_eng._bcast(torch.zeros(_HDR, dtype=torch.long, device=any_eng.cdev))
        cmd = int(hdr0[0])
        if cmd == CMD_STOP:
            return served
        if cmd == CMD_GENERATE:
            payload = []
            for _ in range(int(hdr0[1])):
                hdr = any_eng._bcast(torch.zeros(_HDR, dtype=torch.long, device=any_eng.cdev))
                eng = engines[int(hdr[0])]
                fl = eng._bcast(torch.zeros(4, dtype=torch.float64, device=eng.cdev))
                ids = eng._bcast(torch.zeros(eng.M * eng.b, int(hdr[2]), dtype=torch.long, device=eng.cdev))
                lens = eng._bcast(torch.zeros(eng.M * eng.b, dtype=torch.long, device=eng.cdev))
                payload.append((eng, hdr, fl, ids, lens))
            _run_jobs(payload)
        elif cmd == CMD_SCORE:
            eng = engines[int(hdr0[1])]
            ids = eng._bcast(torch.zeros(int(hdr0[2]), dtype=torch.long, device=eng.cdev))
            eng._run_score(ids)
        elif cmd in (CMD_SLOT_OPEN, CMD_SLOT_ADMIT, CMD_SLOT_STEP):
            handle_slot_command(engines[int(hdr0[1])], hdr0)
        else:
            raise RuntimeError(f"unknown pipeline command {cmd}")
        served += 1


def stop_workers(engine: PipelineGenerator) -> None:
    """Driver: release the workers' serve loop (a second call sends nothing: nobody listens)."""
    if getattr(engine, "_stopped", False):
        return
    engine._stopped = True
    if dist.is_initialized() and dist.get_world_size() > 1 and engine.grank == 0:
        hdr = torch.zeros(_HDR, dtype=torch.long, device=engine.cdev)
        hdr[0] = CMD_STOP
        engine._bcast(hdr)
