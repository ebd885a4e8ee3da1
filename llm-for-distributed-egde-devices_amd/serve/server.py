"""Request-serving engine: a queue of generation requests batched onto one Generator.

The reference serves only a time string (Code/gRPC/server.py, 10 worker threads, stateless).
Here concurrent clients (REST ``POST /generate`` or in-process callers) enqueue requests and one
worker thread serves them, in one of two modes:
  * ``continuous=True`` (default): iteration-level batching (engine.continuous.SlotDecoder) — a
    request is admitted into a free cache slot between decode steps, every step advances all
    occupied slots, a finished request frees its slot at once.  One sampling configuration per
    session (the fused sampler takes one per launch); a request needing another configuration
    waits until the running session drains.
  * ``continuous=False``: static batches — requests with identical sampling settings are grouped
    into batches of up to ``max_batch`` and each batch runs to completion.
Counters and per-token latency percentiles are exposed through ``metrics()``.
"""
from __future__ import annotations

import os
import queue
import threading
import time
from concurrent.futures import Future
from typing import Dict, List, Optional

from ..engine.continuous import SlotDecoder
from ..engine.generate import Generator, SamplingParams
from ..utils.tracing import LatencyHistogram, MetricsWriter, trace_range


class ServingEngine:
    def __init__(self, generator: Generator, tokenizer, max_batch: int = 8, batch_wait_s: float = 0.005,
                 metrics_path: Optional[str] = None, continuous: Optional[bool] = None, steps_per_poll: int = 4):
        self.gen, self.tok = generator, tokenizer
        # one JSONL record per served batch (EDGELLM_METRICS=<path> or metrics_path)
        self.writer = MetricsWriter(metrics_path or os.environ.get("EDGELLM_METRICS"))
        # rows one batch can hold: the cache rows (Generator) or the pipeline's micro-batches x rows
        cap = generator.kv.max_batch if hasattr(generator, "kv") else generator.M * generator.b
        self.max_batch = min(max_batch, cap)
        self.batch_wait_s = batch_wait_s
        self.q: "queue.Queue[tuple]" = queue.Queue()
        self.lat = LatencyHistogram()
        self.stats = {"requests": 0, "batches": 0, "generated_tokens": 0, "errors": 0, "sessions": 0,
                      "decode_steps": 0, "max_concurrent": 0}
        # continuous batching needs per-row cache lengths: not with a HeadInfer-offloaded cache
        # continuous batching drives a Generator's cache rows (not a HeadInfer cache, not a pipeline)
        # (a PipelineGenerator opens its sessions through generator.slot_decoder: parallel.pp_slots)
        slots_ok = getattr(generator, "attn_hook", 1) is None
        self.continuous = slots_ok if continuous is None else (continuous and slots_ok)
        self.width = 2048                          # SlotDecoder output columns per session
        self.steps_per_poll = max(1, steps_per_poll)
        self._closed = False
        self._stop = threading.Event()
        self._worker = threading.Thread(target=self._loop_continuous if self.continuous else self._loop, daemon=True)
        self._worker.start()

    # ------------------------------------------------------------------ API
    def submit(self, prompt_ids: List[int], sampling: SamplingParams, seed: int = 0) -> Future:
        fut: Future = Future()
        err = self.reject_reason(prompt_ids, sampling)
        if err is not None:                        # can never be served: fail now, never queue it
            self.stats["errors"] += 1
            fut.set_exception(ValueError(err))
            return fut
        self.q.put((list(prompt_ids), sampling, seed, fut, time.perf_counter()))
        return fut

    def reject_reason(self, prompt_ids: List[int], sampling: SamplingParams) -> Optional[str]:
        """Why a request can never be admitted (None when it can): an empty prompt, prompt +
        max_new_tokens beyond the cache, or (continuous mode) more new tokens than a session's
        output width."""
        n, new = len(prompt_ids), int(sampling.max_new_tokens)
        if n == 0:
            return "empty prompt"
        if new < 1:
            return "max_new_tokens must be >= 1"
        if n + new > self.gen.max_seq:
            return f"prompt ({n}) + max_new_tokens ({new}) exceeds the cache length {self.gen.max_seq}"
        if self.continuous and new >= self.width:
            return f"max_new_tokens ({new}) must be below the session width {self.width}"
        return None

    def generate_request(self, req: Dict) -> Dict:
        ids = req.get("prompt_ids") or self.tok.encode(req.get("prompt") or "")
        sp = SamplingParams(req.get("max_new_tokens", 64), req.get("temperature", 0.7), req.get("top_k", 50),
                            req.get("top_p", 0.9), req.get("repetition_penalty", 1.1), req.get("do_sample", True))
        out = self.submit(ids, sp, req.get("seed", 0)).result()
        return out

    def metrics(self) -> Dict:
        lat = {k: (None if v != v else v) for k, v in self.lat.summary().items()}   # NaN -> null (JSON)
        return {**self.stats, **lat}

    def close(self):
        """Stop the worker (requests already queued are served first), then release a pipeline
        engine's worker ranks (``shutdown``: their command loop returns and the job exits).
        Idempotent; called from the REST app's shutdown event and at interpreter exit."""
        if self._closed:
            return
        self._closed = True
        self._stop.set()
        self.q.put(None)
        self._worker.join(timeout=600 if getattr(self.gen, "fatal_on_error", False) else 10)
        shutdown = getattr(self.gen, "shutdown", None)
        if shutdown is not None and not self._worker.is_alive():   # never beside a running command
            shutdown()

    def _fatal(self, e: BaseException):
        """A pipeline engine failed after a command went out: the worker ranks are part-way through
        its P2P, so the next command would not line up with them.  Fail the caller(s) and exit the
        process non-zero (torchrun then tears the job down) instead of serving on."""
        import sys
        import traceback
        sys.stderr.write(f"[edgellm serve] fatal pipeline error, exiting: {e!r}\n")
        traceback.print_exc()
        sys.stderr.flush()
        os._exit(70)

    # ------------------------------------------------------------------ continuous worker
    def _loop_continuous(self):
        pending: List[tuple] = []
        dec: Optional[SlotDecoder] = None
        eos = getattr(self.tok, "eos_token_id", None)
        while True:
            stop = self._stop.is_set()
            try:                                   # block only when there is nothing to decode
                item = self.q.get(timeout=0.1) if (not pending and (dec is None or not dec.busy())) \
                    and not stop else self.q.get_nowait()
                if item is None:
                    self._stop.set()
                else:
                    pending.append(item)
                while True:
                    item = self.q.get_nowait()
                    if item is None:
                        self._stop.set()
                    else:
                        pending.append(item)
            except queue.Empty:
                pass
            if self._stop.is_set() and not pending and (dec is None or not dec.busy()):
                break
            try:
                if dec is not None and not dec.busy() and (
                        not pending or pending[0][1].key() != dec.sp.key() or dec.col * 2 > dec.width
                        or not dec.can_admit(len(pending[0][0]), pending[0][1].max_new_tokens)):
                    dec = None                     # session drained: the queue head picks the next one
                if dec is None and pending:
                    factory = getattr(self.gen, "slot_decoder", None)
                    if factory is not None:
                        dec = factory(pending[0][1], seed=pending[0][2], width=self.width, max_batch=self.max_batch)
                    else:
                        dec = SlotDecoder(self.gen, pending[0][1], seed=pending[0][2], width=self.width,
                                          max_batch=self.max_batch)
                    self.stats["sessions"] += 1
                if dec is None:
                    continue
                # admit every waiting request of this session's sampling configuration that fits;
                # a request whose admission fails is failed alone and dropped
                keep, take = [], []
                nfree = len(dec.free_slots())
                for it in pending:
                    ids, sp, _, fut, t_sub = it
                    if sp.key() == dec.sp.key() and len(take) < nfree and dec.can_admit(len(ids), sp.max_new_tokens):
                        take.append(it)
                    else:
                        keep.append(it)
                pending = keep
                if take and hasattr(dec, "admit_batch"):
                    # one command admits them all (pipeline: one ragged prefill per stage)
                    dec.admit_batch([(it[0], it[1].max_new_tokens, eos, it) for it in take])
                else:
                    for it in take:
                        try:
                            dec.admit(it[0], it[1].max_new_tokens, eos, tag=it)
                        except Exception as e:     # noqa: BLE001 - reported to that caller
                            if getattr(self.gen, "fatal_on_error", False):
                                raise
                            self.stats["errors"] += 1
                            if not it[3].done():
                                it[3].set_exception(e)
                if not dec.busy():
                    continue                       # nothing admitted: the head opens a new session
                occ = sum(s is not None for s in dec.slots)
                self.stats["max_concurrent"] = max(self.stats["max_concurrent"], occ)
                n = dec.step(self.steps_per_poll)
                self.stats["decode_steps"] += n
                for it, res in dec.poll():
                    self._finish(it, res, occ)
            except Exception as e:  # fail the requests in flight, keep serving
                self.stats["errors"] += 1
                for s in (dec.slots if dec is not None else []):
                    if s is not None and not s.tag[3].done():
                        s.tag[3].set_exception(e)
                dec = None
                if getattr(self.gen, "fatal_on_error", False):
                    self._fatal(e)

    def _finish(self, it: tuple, res, occ: int):
        toks = res.tokens[0]
        self.stats["requests"] += 1
        self.stats["generated_tokens"] += len(toks)
        if len(toks) > 1 and res.decode_s > 0:
            self.lat.extend([res.decode_s * 1e3 / (len(toks) - 1)])
        self.writer.write(event="request", mode="continuous", prompt_tokens=len(it[0]), generated_tokens=len(toks),
                          ttft_ms=res.prefill_s * 1e3, elapsed_s=res.elapsed_s, slots_busy=occ,
                          queue_ms=(time.perf_counter() - it[4]) * 1e3)
        now = time.perf_counter()
        it[3].set_result({"tokens": toks, "text": self.tok.decode(toks, skip_special_tokens=True),
                          "tokens_per_s": len(toks) / res.elapsed_s if res.elapsed_s > 0 else 0.0,
                          "queue_ms": (now - it[4]) * 1e3, "batch_size": occ,
                          # submission -> first token (queueing + admission prefill)
                          "ttft_ms": ((now - it[4]) - (res.elapsed_s - res.prefill_s)) * 1e3,
                          "latency_ms": (now - it[4]) * 1e3})

    # ------------------------------------------------------------------ static-batch worker
    def _loop(self):
        """Static batches: the queue head's sampling configuration and every waiting request with the
        same one (up to max_batch) run as one generate call.  After close() the requests already
        queued are still served, then the loop exits."""
        pending: List[tuple] = []
        while True:
            if not pending:
                if self._stop.is_set():
                    break
                try:
                    item = self.q.get(timeout=0.1)
                except queue.Empty:
                    continue
                if item is None:
                    self._stop.set()
                    continue
                pending.append(item)
                time.sleep(self.batch_wait_s)      # let concurrent submitters join the batch
            while True:
                try:
                    item = self.q.get_nowait()
                except queue.Empty:
                    break
                if item is None:
                    self._stop.set()
                else:
                    pending.append(item)
            key = pending[0][1]
            batch = [p for p in pending if p[1] == key][: self.max_batch]
            taken = {id(p) for p in batch}
            pending = [p for p in pending if id(p) not in taken]
            self._run(batch)

    def _run(self, batch: List[tuple]):
        prompts = [b[0] for b in batch]
        sp = batch[0][1]
        try:
            with trace_range(f"serve.batch{len(batch)}"):
                res = self.gen.generate(prompts, sp, seed=batch[0][2],
                                        eos_token_id=getattr(self.tok, "eos_token_id", None))
        except Exception as e:  # report to every caller, keep serving
            self.stats["errors"] += 1
            for b in batch:
                b[3].set_exception(e)
            if getattr(self.gen, "fatal_on_error", False):
                self._fatal(e)
            return
        self.stats["batches"] += 1
        steps = max((len(t) for t in res.tokens), default=0)
        self.lat.extend(res.step_ms or ([res.elapsed_s * 1e3 / steps] if steps else []))
        step = sorted(res.step_ms)
        self.writer.write(event="batch", batch_size=len(batch), prompt_tokens=sum(len(p) for p in prompts),
                          generated_tokens=sum(len(t) for t in res.tokens), ttft_ms=res.prefill_s * 1e3,
                          elapsed_s=res.elapsed_s, p50_step_ms=step[len(step) // 2] if step else None,
                          max_queue_ms=max((time.perf_counter() - b[4]) * 1e3 for b in batch))
        for i, b in enumerate(batch):
            toks = res.tokens[i]
            self.stats["requests"] += 1
            self.stats["generated_tokens"] += len(toks)
            b[3].set_result({"tokens": toks, "text": self.tok.decode(toks, skip_special_tokens=True),
                             "tokens_per_s": len(toks) / res.elapsed_s if res.elapsed_s > 0 else 0.0,
                             "queue_ms": (time.perf_counter() - b[4]) * 1e3, "batch_size": len(batch)})
