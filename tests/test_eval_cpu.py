"""Metric harness against hand-computed values, and the ensemble merges with stub agents
(SURVEY §4 items 5-6).  rouge_score / nltk / sacrebleu are not installed here, so the expected
numbers are derived by hand from the metric definitions the reference uses
(combine_model_fp_updated.py:46-73: rouge_scorer with use_stemmer=True, HF evaluate "bleu")."""
import math
from types import SimpleNamespace

import pytest
import torch

from edgellm.engine import SamplingParams
from edgellm.eval.porter import stem
from edgellm.eval.text_metrics import corpus_bleu, evaluate_bleu, evaluate_rouge, mean_rouge, rouge_scores
from edgellm.orchestrator.ensemble import Orchestrator, RefineMerge, VoteMerge
from edgellm.orchestrator.prompts import QA_TEMPLATE, qa_prompt, refine_prompt


def test_rouge_hand_computed():
    # unigrams: 5 of 6 match both ways; bigrams: the-cat, on-the, the-mat = 3 of 5; LCS = 5
    r1, r2, rl = evaluate_rouge("the cat is on the mat", "the cat sat on the mat")
    assert r1 == pytest.approx(5 / 6) and r2 == pytest.approx(3 / 5) and rl == pytest.approx(5 / 6)
    assert mean_rouge(r1, r2, rl) == pytest.approx((5 / 6 + 3 / 5 + 5 / 6) / 3)
    # stemming (use_stemmer=True): runs/running -> run, dogs -> dog; P = 2/2, R = 2/3
    s = rouge_scores("running dogs", "the dog runs")
    assert s["rouge1"][0] == pytest.approx(1.0) and s["rouge1"][1] == pytest.approx(2 / 3)
    assert s["rouge1"][2] == pytest.approx(0.8)
    assert evaluate_rouge("", "anything") == (0.0, 0.0, 0.0)


def test_porter_stemmer_reference_cases():
    cases = {"caresses": "caress", "ponies": "poni", "running": "run", "relational": "relat",
             "hopping": "hop", "generalization": "gener", "agreed": "agre", "sky": "sky"}
    for w, s in cases.items():
        assert stem(w) == s, (w, stem(w), s)


def test_bleu_hand_computed():
    assert evaluate_bleu("the quick brown fox jumps", "the quick brown fox jumps") == pytest.approx(1.0)
    # all n-gram precisions 1, brevity penalty exp(1 - 6/5)
    assert evaluate_bleu("a b c d e", "a b c d e f") == pytest.approx(math.exp(-0.2))
    # no 4-gram match and no smoothing -> 0 (HF evaluate default)
    assert evaluate_bleu("a b c x d e", "a b c d e f") == 0.0
    out = corpus_bleu(["a b c d e"], [["a b c d e f"]])
    assert out["precisions"] == [1.0, 1.0, 1.0, 1.0] and out["reference_length"] == 6


def _res(tps=10.0):
    return SimpleNamespace(tps_generated=lambda: tps)


class StubAgent:
    """Duck-typed Agent: fixed answer, records the prompt it was given."""

    def __init__(self, name, answer, device="cpu", tps=10.0):
        self.name, self.answer, self.cpu_prompt = name, answer, False
        self.device = torch.device(device)
        self.sampling = SamplingParams(max_new_tokens=16)
        self.prompts, self.tps = [], tps

    def run(self, prompt_text, seed, legacy_decode=True, sampling=None):
        self.prompts.append((prompt_text, sampling))
        return self.answer, _res(self.tps)


def test_vote_merge_majority_and_medoid():
    vote = VoteMerge()
    final, _ = vote({"a": "Paris is the capital", "b": "paris  is the CAPITAL", "c": "Lyon"}, "q", None, 0)
    assert final == "Paris is the capital"
    # no majority: the answer with the highest summed ROUGE-L to the others wins
    final, _ = vote({"a": "the capital of france is paris", "b": "paris is the capital of france",
                     "c": "bananas are yellow"}, "q", None, 0)
    assert final in ("the capital of france is paris", "paris is the capital of france")


def test_orchestrator_refine_uses_reference_prompt_and_tps_rules():
    a1, a2 = StubAgent("phi", "Answer one.", tps=10.0), StubAgent("pythia", "Answer two.", tps=30.0)
    ref = StubAgent("refiner", "Refined.", tps=99.0)
    orch = Orchestrator([a1, a2], RefineMerge(ref), concurrent=False)
    out = orch.answer("What is the capital of France?", reference="Paris", seed=3)
    assert out.final == "Refined." and out.answers == {"phi": "Answer one.", "pythia": "Answer two."}
    assert a1.prompts[0][0] == qa_prompt("What is the capital of France?")
    assert a1.prompts[0][0].startswith(QA_TEMPLATE.split("{")[0])
    rprompt, rsp = ref.prompts[0]
    assert rprompt == refine_prompt(["Answer one.", "Answer two."], "Paris")
    assert "Reference (optional):\nParis" in rprompt                   # the reference's leak, kept
    assert (rsp.temperature, rsp.top_k, rsp.top_p, rsp.repetition_penalty) == (0.5, 30, 0.9, 1.1)
    # Combo TPS = mean of the QA agents only (combine_model_fp_updated.py:209)
    assert out.combo_tps == pytest.approx(20.0) and out.tps["merger"] == 99.0
    no_leak = RefineMerge(ref, include_reference=False)
    no_leak({"a": "x", "b": "y"}, "q", "Paris", 0)
    assert "Paris" not in ref.prompts[-1][0]


def test_orchestrator_runs_agents_concurrently_on_distinct_devices():
    import threading
    meet = threading.Barrier(3, timeout=10)           # only passes if all three run at once

    class Tracking(StubAgent):
        def run(self, *a, **k):
            meet.wait()
            return super().run(*a, **k)

    agents = [Tracking("x", "same"), Tracking("y", "same"), Tracking("z", "other")]
    agents[1].device = torch.device("meta")           # distinct "device groups" -> threads
    out = Orchestrator(agents, VoteMerge(), concurrent=True).answer("q")
    assert out.final == "same" and out.merge == "vote"


def test_confidence_scores_batched_equals_per_text():
    """One right-padded scorer pass per group of texts gives each text's own confidence."""
    from edgellm.eval.metrics import confidence_score, confidence_scores
    from edgellm.models import build_model, tiny
    m = build_model(tiny("llama"), dtype=torch.float32, seed=3)
    texts = [[5, 9, 2, 7], [1], [], [3, 3, 8, 1, 4, 4, 2, 9, 9], [6, 2]]
    got = confidence_scores(m, texts, rows_per_pass=3)
    want = [confidence_score(m, t) for t in texts]
    assert got == pytest.approx(want, abs=1e-5)
