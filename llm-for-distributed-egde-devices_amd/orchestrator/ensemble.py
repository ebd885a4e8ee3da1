"""Multi-agent ensemble: N QA agents + a merge step.

Reference flow (combine_model_fp_updated.py:188-221): Phi-2 answers, then Pythia-1B answers,
then Llama-3.2-1B-Instruct "refines" both answers — strictly in series in one process.
Here agents are independent engines on their own devices and run CONCURRENTLY (one host thread
per agent; the decode loops are graph replays, so the GIL is not the bottleneck); the merge
waits for all of them.  Merges:
  * ``RefineMerge`` — the reference's LLM refiner (prompt with every answer + optional gold
    reference, fixed sampling T=0.5, top-k 30, top-p 0.9, rep 1.1: combine_model_fp_updated.py:128-132)
  * ``VoteMerge``   — majority vote (north star): the answer most agents agree on (normalised
    exact match), else the medoid under ROUGE-L F1 agreement
Decoding follows the reference by default (``legacy_decode_includes_prompt``: the decoded text
contains the prompt, combine_model_fp_updated.py:109,135); switch it off to score answers only.
TPS: combo = mean of the QA agents' generated-token TPS (refiner excluded, :209) or of all
agents (the CPU script's definition, try.py:323).
"""
from __future__ import annotations

import threading
import time
from collections import Counter
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import torch

from ..config import REFINER_SAMPLING
from ..engine.generate import GenerationResult, Generator, SamplingParams
from ..eval.text_metrics import rouge_scores
from .prompts import qa_prompt, refine_prompt


@dataclass
class Agent:
    name: str
    generator: Generator
    tokenizer: object
    sampling: SamplingParams
    cpu_prompt: bool = False

    @property
    def device(self):
        return self.generator.device

    def run(self, prompt_text: str, seed: int, legacy_decode: bool = True, sampling: Optional[SamplingParams] = None):
        sp = sampling or self.sampling
        ids = self.tokenizer.encode(prompt_text)
        max_seq = self.generator.max_seq
        if len(ids) + sp.max_new_tokens > max_seq:                  # truncation=True semantics
            ids = ids[-(max_seq - sp.max_new_tokens):]
        eos = getattr(self.tokenizer, "eos_token_id", None)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        res = self.generator.generate([ids], sp, seed=seed, eos_token_id=eos)
        toks = res.tokens[0]
        text = self.tokenizer.decode((ids + toks) if legacy_decode else toks, skip_special_tokens=True).strip()
        return text, res

    def run_batch(self, prompt_texts: Sequence[str], seed: int, legacy_decode: bool = True,
                  sampling: Optional[SamplingParams] = None):
        """Decode several prompts together (one batched generate: per-sequence prefill, one
        graph-replayed decode step for all rows).  Returns (texts, GenerationResult)."""
        sp = sampling or self.sampling
        max_seq = self.generator.max_seq
        ids_list = []
        for t in prompt_texts:
            ids = self.tokenizer.encode(t)
            if len(ids) + sp.max_new_tokens > max_seq:
                ids = ids[-(max_seq - sp.max_new_tokens):]
            ids_list.append(ids)
        eos = getattr(self.tokenizer, "eos_token_id", None)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        res = self.generator.generate(ids_list, sp, seed=seed, eos_token_id=eos)
        texts = [self.tokenizer.decode((ids + toks) if legacy_decode else toks, skip_special_tokens=True).strip()
                 for ids, toks in zip(ids_list, res.tokens)]
        return texts, res


@dataclass
class EnsembleResult:
    question: str
    answers: Dict[str, str]
    final: str
    results: Dict[str, GenerationResult]
    tps: Dict[str, float]
    combo_tps: float
    wall_s: float
    merge: str


class VoteMerge:
    name = "vote"

    @staticmethod
    def _norm(s: str) -> str:
        return " ".join(s.lower().split())

    def __call__(self, answers: Dict[str, str], question: str, reference: Optional[str], seed: int):
        texts = list(answers.values())
        counts = Counter(self._norm(t) for t in texts)
        top, n = counts.most_common(1)[0]
        if n > len(texts) / 2:
            return next(t for t in texts if self._norm(t) == top), None
        best, best_score = texts[0], -1.0
        for i, a in enumerate(texts):
            s = sum(rouge_scores(a, b)["rougeL"][2] for j, b in enumerate(texts) if j != i)
            if s > best_score:
                best, best_score = a, s
        return best, None


class RefineMerge:
    name = "refine"

    def __init__(self, refiner: Agent, include_reference: bool = True, legacy_decode: bool = True):
        self.refiner, self.include_reference, self.legacy_decode = refiner, include_reference, legacy_decode

    def _sampling(self):
        return SamplingParams(max_new_tokens=self.refiner.sampling.max_new_tokens, **REFINER_SAMPLING)

    def __call__(self, answers: Dict[str, str], question: str, reference: Optional[str], seed: int):
        prompt = refine_prompt(list(answers.values()), reference, self.include_reference)
        text, res = self.refiner.run(prompt, seed, self.legacy_decode, self._sampling())
        return text, res

    def batch(self, answers: List[Dict[str, str]], questions, references, seed: int):
        prompts = [refine_prompt(list(a.values()), r, self.include_reference) for a, r in zip(answers, references)]
        texts, res = self.refiner.run_batch(prompts, seed, self.legacy_decode, self._sampling())
        return texts, res


class Orchestrator:
    def __init__(self, agents: Sequence[Agent], merge, concurrent: bool = True, legacy_decode: bool = True,
                 tps_includes_merger: bool = False):
        self.agents = list(agents)
        self.merge = merge
        self.concurrent = concurrent
        self.legacy_decode = legacy_decode
        self.tps_includes_merger = tps_includes_merger

    def answer(self, question: str, reference: Optional[str] = None, seed: int = 0) -> EnsembleResult:
        t0 = time.perf_counter()
        answers: Dict[str, str] = {}
        results: Dict[str, GenerationResult] = {}
        errors: List[BaseException] = []

        def work(i, agent):
            try:
                text, res = agent.run(qa_prompt(question, agent.cpu_prompt), seed + 1000 * i, self.legacy_decode)
                answers[agent.name], results[agent.name] = text, res
            except BaseException as e:  # surfaced after join
                errors.append(e)

        devices = {a.device for a in self.agents}
        if self.concurrent and len(self.agents) > 1 and len(devices) > 1:
            threads = [threading.Thread(target=work, args=(i, a)) for i, a in enumerate(self.agents)]
            for t in threads:
                t.start()
            for t in threads:
                t.join()
        else:
            for i, a in enumerate(self.agents):
                work(i, a)
        if errors:
            raise errors[0]
        ordered = {a.name: answers[a.name] for a in self.agents}
        final, mres = self.merge(ordered, question, reference, seed)
        tps = {n: r.tps_generated() for n, r in results.items()}
        vals = list(tps.values())
        if mres is not None:
            tps["merger"] = mres.tps_generated()
            if self.tps_includes_merger:
                vals.append(tps["merger"])
        return EnsembleResult(question, ordered, final, results, tps, sum(vals) / len(vals), time.perf_counter() - t0,
                              getattr(self.merge, "name", "custom"))

    def answer_batch(self, questions: Sequence[str], references: Sequence[Optional[str]], seed: int = 0
                     ) -> List[EnsembleResult]:
        """Batched ``answer``: every agent decodes all questions of the batch together (agents on
        distinct devices concurrently), then the merge runs batched (refiner) or per question
        (vote).  Per-sample TPS = the sample's generated tokens / its agent's batch wall time (a
        per-stream rate, comparable with the reference's batch-1 TPS); the batch's aggregate
        throughput is ``sum(generated) / wall``."""
        t0 = time.perf_counter()
        outs: Dict[str, tuple] = {}
        errors: List[BaseException] = []

        def work(i, agent):
            try:
                prompts = [qa_prompt(q, agent.cpu_prompt) for q in questions]
                outs[agent.name] = agent.run_batch(prompts, seed + 1000 * i, self.legacy_decode)
            except BaseException as e:  # surfaced after join
                errors.append(e)

        devices = {a.device for a in self.agents}
        if self.concurrent and len(self.agents) > 1 and len(devices) > 1:
            threads = [threading.Thread(target=work, args=(i, a)) for i, a in enumerate(self.agents)]
            for t in threads:
                t.start()
            for t in threads:
                t.join()
        else:
            for i, a in enumerate(self.agents):
                work(i, a)
        if errors:
            raise errors[0]
        n = len(questions)
        answers = [{a.name: outs[a.name][0][j] for a in self.agents} for j in range(n)]
        per_tps = [{a.name: len(outs[a.name][1].tokens[j]) / max(outs[a.name][1].elapsed_s, 1e-9) for a in self.agents}
                   for j in range(n)]
        if hasattr(self.merge, "batch"):
            finals, mres = self.merge.batch(answers, questions, references, seed)
            for j in range(n):
                per_tps[j]["merger"] = len(mres.tokens[j]) / max(mres.elapsed_s, 1e-9)
        else:
            finals = [self.merge(answers[j], questions[j], references[j], seed)[0] for j in range(n)]
        wall = time.perf_counter() - t0
        out = []
        for j in range(n):
            tps = per_tps[j]
            vals = [v for k, v in tps.items() if k != "merger" or self.tps_includes_merger]
            out.append(EnsembleResult(questions[j], answers[j], finals[j],
                                      {a.name: outs[a.name][1] for a in self.agents}, tps, sum(vals) / len(vals),
                                      wall / n, getattr(self.merge, "name", "custom")))
        return out
