"""Request-serving engine: a queue of generation requests batched onto one Generator.

The reference serves only a time string (Code/gRPC/server.py, 10 worker threads, stateless).
Here concurrent clients (REST ``POST /generate`` or in-process callers) enqueue requests; one
worker thread drains the queue, groups requests with identical sampling settings into batches
of up to ``max_batch`` (the fused sampler takes one configuration per launch) and runs them
through the graph-captured decode loop.  Counters and per-token latency percentiles are exposed
through ``metrics()``.
"""
from __future__ import annotations

import os
import queue
import threading
import time
from concurrent.futures import Future
from typing import Dict, List, Optional

from ..engine.generate import Generator, SamplingParams
from ..utils.tracing import LatencyHistogram, MetricsWriter, trace_range


class ServingEngine:
    def __init__(self, generator: Generator, tokenizer, max_batch: int = 8, batch_wait_s: float = 0.005,
                 metrics_path: Optional[str] = None):
        self.gen, self.tok = generator, tokenizer
        # one JSONL record per served batch (EDGELLM_METRICS=<path> or metrics_path)
        self.writer = MetricsWriter(metrics_path or os.environ.get("EDGELLM_METRICS"))
        self.max_batch = min(max_batch, generator.kv.max_batch)
        self.batch_wait_s = batch_wait_s
        self.q: "queue.Queue[tuple]" = queue.Queue()
        self.lat = LatencyHistogram()
        self.stats = {"requests": 0, "batches": 0, "generated_tokens": 0, "errors": 0}
        self._stop = threading.Event()
        self._worker = threading.Thread(target=self._loop, daemon=True)
        self._worker.start()

    # ------------------------------------------------------------------ API
    def submit(self, prompt_ids: List[int], sampling: SamplingParams, seed: int = 0) -> Future:
        fut: Future = Future()
        self.q.put((list(prompt_ids), sampling, seed, fut, time.perf_counter()))
        return fut

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
        self._stop.set()
        self.q.put(None)
        self._worker.join(timeout=10)

    # ------------------------------------------------------------------ worker
    def _loop(self):
        pending: List[tuple] = []
        while not self._stop.is_set():
            try:
                item = self.q.get(timeout=0.1) if not pending else self.q.get_nowait()
                if item is None:
                    break
                pending.append(item)
                continue
            except queue.Empty:
                pass
            if not pending:
                continue
            time.sleep(self.batch_wait_s)          # let concurrent submitters join the batch
            while True:
                try:
                    item = self.q.get_nowait()
                except queue.Empty:
                    break
                if item is None:
                    self._stop.set()
                    break
                pending.append(item)
            key = pending[0][1]
            batch = [p for p in pending if p[1] == key][: self.max_batch]
            pending = [p for p in pending if p not in batch]
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
