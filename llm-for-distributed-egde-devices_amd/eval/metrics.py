"""The reference's nine per-sample metrics and their aggregation.

Per sample (combine_model_fp_updated.py:203-212): ROUGE-1/2/L F1, BERTScore F1, BLEU, cosine
similarity of sentence embeddings, confidence (an extra forward pass of the scoring LM:
mean over positions of the max softmax probability — K13, here the fused
``ops.max_softmax_prob`` kernel), and tokens/sec.  Error policy = the reference's: any metric
exception zeroes every metric of that sample, TPS included (``strict=True`` raises instead).
Progress can be appended to a JSONL file and resumed (the reference restarts all 1000 samples
after a crash — SURVEY §5.4).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops
from ..engine.kv_cache import KVCache
from ..models.decoder import AttnCtx, DecoderLM
from .text_metrics import evaluate_bleu, evaluate_rouge

METRIC_KEYS = ("rouge1", "rouge2", "rougeL", "bertscore", "bleu", "cosine", "confidence", "tps")


@torch.no_grad()
def confidence_score(model: DecoderLM, ids: List[int]) -> float:
    """mean_t max_v softmax(logits[t])  over the text's own tokens (one prefill pass).  A
    pipeline-parallel scorer (parallel/pp_engine.py) runs that pass through its stages."""
    if not ids:
        return 0.0
    if hasattr(model, "confidence"):
        return float(model.confidence(ids))
    dev = model.device
    T = len(ids)
    kv = KVCache(model.cfg, 1, T, dtype=model.dtype, device=dev)
    sp = torch.zeros(1, dtype=torch.int32, device=dev)
    ctx = AttnCtx("prefill", 1, T, sp, sp + T, T, kv, model.rope_table(dev))
    logits = model(torch.tensor([ids], device=dev), ctx, logits="all")
    return float(ops.max_softmax_prob(logits).mean())


@torch.no_grad()
def confidence_scores(model: DecoderLM, ids_list: List[List[int]], rows_per_pass: int = 32) -> List[float]:
    """``confidence_score`` of several texts with one right-padded prefill pass per
    ``rows_per_pass`` texts (causal attention: a real token never sees the pads, so each row's
    per-token logits are its own pass's); pads are excluded from each row's mean."""
    if hasattr(model, "confidence") or not ids_list:
        return [confidence_score(model, ids) for ids in ids_list]
    out: List[float] = [0.0] * len(ids_list)
    dev = model.device
    live = [i for i, ids in enumerate(ids_list) if ids]
    for c0 in range(0, len(live), rows_per_pass):
        idx = live[c0:c0 + rows_per_pass]
        B, T = len(idx), max(len(ids_list[i]) for i in idx)
        x = torch.zeros(B, T, dtype=torch.long)
        for r, i in enumerate(idx):
            x[r, :len(ids_list[i])] = torch.tensor(ids_list[i])
        kv = KVCache(model.cfg, B, T, dtype=model.dtype, device=dev)
        sp = torch.zeros(B, dtype=torch.int32, device=dev)
        ctx = AttnCtx("prefill", B, T, sp, sp + T, T, kv, model.rope_table(dev))
        logits = model(x.to(dev), ctx, logits="all")
        p = ops.max_softmax_prob(logits).float().view(B, T).cpu()
        for r, i in enumerate(idx):
            out[i] = float(p[r, :len(ids_list[i])].mean())
    return out


class Embedder:
    """Sentence embeddings + contextual token embeddings from a BERT-style encoder."""

    def __init__(self, encoder, tokenizer, device=None, max_len: int = 256):
        self.enc, self.tok, self.device, self.max_len = encoder, tokenizer, device, max_len

    def _ids(self, text: str) -> torch.Tensor:
        ids = self.tok.encode(text)[: self.max_len]
        vmax = self.enc.cfg.vocab_size
        return torch.tensor([[i % vmax for i in ids] or [0]], device=self.device)

    @torch.no_grad()
    def sentence(self, text: str) -> torch.Tensor:
        return self.enc.sentence_embedding(self._ids(text))[0]

    @torch.no_grad()
    def tokens(self, text: str) -> torch.Tensor:
        return self.enc(self._ids(text))[0].float()


def cosine_similarity(pred: str, ref: str, embedder: Embedder) -> float:
    """util.pytorch_cos_sim of the two sentence embeddings (combine_model_fp_updated.py:70-73)."""
    return float(F.cosine_similarity(embedder.sentence(pred), embedder.sentence(ref), dim=0))


def bertscore_f1(pred: str, ref: str, embedder: Embedder) -> float:
    """BERTScore F1 (greedy max-cosine matching, no idf, no baseline rescale — evaluate's
    defaults).  Parity with roberta-large scores needs that checkpoint: "parity unpinned"."""
    p = F.normalize(embedder.tokens(pred), dim=-1)
    r = F.normalize(embedder.tokens(ref), dim=-1)
    sim = r @ p.t()
    rec = sim.max(1).values.mean()
    prec = sim.max(0).values.mean()
    return float(2 * prec * rec / (prec + rec)) if float(prec + rec) > 0 else 0.0


@dataclass
class MetricSuite:
    embedder: Optional[Embedder] = None
    bert_embedder: Optional[Embedder] = None
    strict: bool = False

    def score(self, pred: str, ref: str, scorer: Optional[DecoderLM] = None, scorer_tok=None,
              tps: float = 0.0, confidence: Optional[float] = None) -> Dict[str, float]:
        """``confidence``: precomputed (``confidence_scores`` over a batch), else one scorer pass."""
        try:
            r1, r2, rl = evaluate_rouge(pred, ref)
            bs = bertscore_f1(pred, ref, self.bert_embedder or self.embedder) if (self.bert_embedder or self.embedder) else 0.0
            bl = evaluate_bleu(pred, ref)
            cs = cosine_similarity(pred, ref, self.embedder) if self.embedder else 0.0
            conf = confidence if confidence is not None else \
                (confidence_score(scorer, scorer_tok.encode(pred)) if scorer is not None else 0.0)
            return dict(rouge1=r1, rouge2=r2, rougeL=rl, bertscore=bs, bleu=bl, cosine=cs, confidence=conf, tps=tps)
        except Exception:
            if self.strict:
                raise
            return {k: 0.0 for k in METRIC_KEYS}


@dataclass
class Results:
    rows: List[Dict[str, float]] = field(default_factory=list)

    def add(self, row: Dict[str, float]):
        self.rows.append(row)

    def means(self) -> Dict[str, float]:
        return {k: float(np.mean([r.get(k, 0.0) for r in self.rows])) if self.rows else 0.0 for k in METRIC_KEYS}


class ProgressLog:
    """Append-only JSONL of per-sample results; ``done()`` lists finished indices for resume."""

    def __init__(self, path: Optional[str]):
        self.path = path

    def done(self) -> Dict[int, dict]:
        out = {}
        if self.path and os.path.exists(self.path):
            with open(self.path) as f:
                for line in f:
                    line = line.strip()
                    if line:
                        rec = json.loads(line)
                        out[int(rec["index"])] = rec
        return out

    def append(self, index: int, rec: dict):
        if not self.path:
            return
        with open(self.path, "a") as f:
            f.write(json.dumps({"index": index, **rec}) + "\n")


class EfficiencyMeter:
    """Table-3 efficiency columns (ACL.pdf p.7) measured by the harness itself:
    "Time Taken" = wall time per sample of the whole loop, metrics included (the reference reads
    tqdm's s/it, Llama_bf16_updated.py:103-124), aggregate generated tok/s of the QA agents, and
    peak device memory (the reference read nvidia-smi by hand; here max_memory_allocated summed
    over the agents' distinct GPUs)."""

    def __init__(self, devices=()):
        import time as _t
        self.devices = sorted({str(d) for d in devices if str(d).startswith("cuda")})
        self.wall = 0.0
        self.n = 0
        self.tokens = 0
        self._t0 = _t.perf_counter()

    def add(self, wall_s: float, n_samples: int, gen_tokens: int):
        self.wall += wall_s
        self.n += n_samples
        self.tokens += gen_tokens

    def peak_gb(self) -> float:
        import torch
        if not self.devices or not torch.cuda.is_available():
            return 0.0
        return sum(torch.cuda.max_memory_allocated(torch.device(d)) for d in self.devices) / 1e9

    def summary(self) -> dict:
        return {"time_per_sample_s": self.wall / max(self.n, 1), "total_time_s": self.wall,
                "agg_tokens_per_s": self.tokens / self.wall if self.wall > 0 else 0.0,
                "peak_mem_gb": self.peak_gb(), "samples": self.n}
