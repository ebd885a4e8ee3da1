"""Multi-agent ensemble: N QA agents + a merge step.

Reference flow (combine_model_fp_updated.py:188-221): Phi-2 answers, then Pythia-1B answers,
then Llama-3.2-1B-Instruct "refines" both answers — strictly in series in one process.
Here agents are independent engines and run CONCURRENTLY: agents on different devices in their
own host threads (the decode loops are graph replays, so the GIL is not the bottleneck), agents
sharing a GPU on their own HIP streams from one thread (``run_agents`` -> engine co_generate);
the merge waits for all of them.  Merges:
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
from ..engine.generate import GenerationResult, Generator, SamplingParams, co_generate
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

    def encode_batch(self, prompt_texts: Sequence[str], sampling: Optional[SamplingParams] = None):
        """Token ids of each prompt, left-truncated so prompt + max_new_tokens fits the cache."""
        sp = sampling or self.sampling
        max_seq = self.generator.max_seq
        ids_list = []
        for t in prompt_texts:
            ids = self.tokenizer.encode(t)
            if len(ids) + sp.max_new_tokens > max_seq:
                ids = ids[-(max_seq - sp.max_new_tokens):]
            ids_list.append(ids)
        return ids_list

    def decode_batch(self, ids_list, res: GenerationResult, legacy_decode: bool = True) -> List[str]:
        return [self.tokenizer.decode((ids + toks) if legacy_decode else toks, skip_special_tokens=True).strip()
                for ids, toks in zip(ids_list, res.tokens)]

    def run_batch(self, prompt_texts: Sequence[str], seed: int, legacy_decode: bool = True,
                  sampling: Optional[SamplingParams] = None):
        """Decode several prompts together (one batched generate: per-sequence prefill, one
        graph-replayed decode step for all rows).  Returns (texts, GenerationResult)."""
        sp = sampling or self.sampling
        ids_list = self.encode_batch(prompt_texts, sp)
        eos = getattr(self.tokenizer, "eos_token_id", None)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        res = self.generator.generate(ids_list, sp, seed=seed, eos_token_id=eos)
        return self.decode_batch(ids_list, res, legacy_decode), res


def run_agents(agents: Sequence[Agent], prompts: Sequence[Sequence[str]], seeds: Sequence[int],
               legacy_decode: bool = True, concurrent: bool = True, single: bool = False) -> List[tuple]:
    """Run agent i on ``prompts[i]`` (a batch of texts) with ``seeds[i]``; returns [(texts, result)].
    Agents on DIFFERENT devices run in parallel host threads; agents sharing a GPU decode side by
    side on their own HIP streams (engine.generate.co_generate) — not one after another.
    ``single``: one prompt per agent through ``Agent.run`` (the batch-1 reference flow)."""
    out: List[Optional[tuple]] = [None] * len(agents)
    errors: List[BaseException] = []
    units: List[List[int]] = []
    shared: Dict[object, List[int]] = {}
    # pipeline agents (one process per GPU under torchrun, parallel/pp_engine.py): one concurrent
    # command for all of them — agents on disjoint rank groups decode at the same time, the rest in
    # order.  Dispatch is on the engine's capability, never on its device type: co_generate drives
    # a plain Generator's internals (start / step / precapture), which a pipeline engine lacks.
    pipe = [i for i, a in enumerate(agents) if _is_pipeline(getattr(a, "generator", None))]
    if pipe:
        _run_pipeline_agents(agents, pipe, prompts, seeds, legacy_decode, concurrent, out)
    for i, a in enumerate(agents):
        if i in pipe:
            continue
        dev = getattr(a, "device", None)
        if concurrent and _is_local_generator(getattr(a, "generator", None)) and isinstance(dev, torch.device) \
                and dev.type == "cuda":
            if dev not in shared:
                shared[dev] = []
                units.append(shared[dev])
            shared[dev].append(i)
        else:
            units.append([i])

    def work(idx):
        try:
            dev = agents[idx[0]].device
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
            if len(idx) > 1:
                jobs, enc = [], []
                for i in idx:
                    a = agents[i]
                    ids = a.encode_batch(prompts[i])
                    enc.append(ids)
                    jobs.append((a.generator, ids, a.sampling, seeds[i], getattr(a.tokenizer, "eos_token_id", None)))
                for i, ids, res in zip(idx, enc, co_generate(jobs)):
                    out[i] = (agents[i].decode_batch(ids, res, legacy_decode), res)
            else:
                for i in idx:
                    if single:
                        text, res = agents[i].run(prompts[i][0], seeds[i], legacy_decode)
                        out[i] = ([text], res)
                    else:
                        out[i] = agents[i].run_batch(prompts[i], seeds[i], legacy_decode)
        except BaseException as e:  # surfaced after join
            errors.append(e)

    devices = {getattr(agents[u[0]], "device", None) for u in units}
    if concurrent and len(units) > 1 and len(devices) > 1:
        threads = [threading.Thread(target=work, args=(idx,)) for idx in units]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
    else:
        for idx in units:
            work(idx)
    if errors:
        raise errors[0]
    return out


def _is_pipeline(gen) -> bool:
    """A multi-process pipeline engine (parallel.pp_engine.PipelineGenerator)."""
    from ..parallel.pp_engine import PipelineGenerator
    return isinstance(gen, PipelineGenerator)


def _is_local_generator(gen) -> bool:
    """An in-process engine that co_generate can drive side by side with others on one GPU."""
    return isinstance(gen, Generator) and all(hasattr(gen, a) for a in ("start", "step", "precapture", "collect"))


def _run_pipeline_agents(agents, idx, prompts, seeds, legacy_decode, concurrent, out):
    from ..parallel.pp_engine import generate_concurrent
    encs = [agents[i].encode_batch(prompts[i]) for i in idx]
    jobs = [(agents[i].generator, ids, agents[i].sampling, seeds[i], getattr(agents[i].tokenizer, "eos_token_id", None))
            for i, ids in zip(idx, encs)]
    results = generate_concurrent(jobs) if concurrent else [r for j in jobs for r in generate_concurrent([j])]
    for i, ids, res in zip(idx, encs, results):
        out[i] = (agents[i].decode_batch(ids, res, legacy_decode), res)


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
        outs = run_agents(self.agents, [[qa_prompt(question, a.cpu_prompt)] for a in self.agents],
                          [seed + 1000 * i for i in range(len(self.agents))], self.legacy_decode, self.concurrent,
                          single=True)
        answers = {a.name: o[0][0] for a, o in zip(self.agents, outs)}
        results = {a.name: o[1] for a, o in zip(self.agents, outs)}
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
        res = run_agents(self.agents, [[qa_prompt(q, a.cpu_prompt) for q in questions] for a in self.agents],
                         [seed + 1000 * i for i in range(len(self.agents))], self.legacy_decode, self.concurrent)
        outs: Dict[str, tuple] = {a.name: o for a, o in zip(self.agents, res)}
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
