"""ROUGE-1/2/L and BLEU with the reference's semantics.

ROUGE  = ``rouge_score.RougeScorer(['rouge1','rouge2','rougeL'], use_stemmer=True).score(ref, pred)``
         F-measures (combine_model_fp_updated.py:46,51-53): lowercase, non-[a-z0-9] -> space,
         Porter-stem tokens longer than 3 characters; ROUGE-N clipped n-gram overlap,
         ROUGE-L longest common subsequence; F1 = 2PR / (P + R).
Mean   = (R1 + R2 + RL) / 3 (combine_model_fp_updated.py:56-57).
BLEU   = ``evaluate.load("bleu").compute(predictions=[pred], references=[[ref]])["bleu"]``
         (combine_model_fp_updated.py:65-67): corpus BLEU, max order 4, no smoothing, brevity
         penalty exp(1 - r/c) for c < r, tokenizer "13a" (sacrebleu's mteval-v13a rules).
"""
from __future__ import annotations

import math
import re
from collections import Counter
from typing import Dict, List, Sequence, Tuple

from .porter import stem

_NON_ALNUM = re.compile(r"[^a-z0-9]+")
_TOKEN_OK = re.compile(r"^[a-z0-9]+$")


def rouge_tokenize(text: str, use_stemmer: bool = True) -> List[str]:
    text = _NON_ALNUM.sub(" ", text.lower())
    toks = [t for t in re.split(r"\s+", text) if t]
    if use_stemmer:
        toks = [stem(t) if len(t) > 3 else t for t in toks]
    return [t for t in toks if _TOKEN_OK.match(t)]


def _ngrams(toks: Sequence[str], n: int) -> Counter:
    return Counter(tuple(toks[i:i + n]) for i in range(len(toks) - n + 1))


def _f1(overlap: float, n_pred: int, n_ref: int) -> Tuple[float, float, float]:
    p = overlap / n_pred if n_pred > 0 else 0.0
    r = overlap / n_ref if n_ref > 0 else 0.0
    f = 2 * p * r / (p + r) if p + r > 0 else 0.0
    return p, r, f


def _lcs(a: Sequence[str], b: Sequence[str]) -> int:
    if not a or not b:
        return 0
    prev = [0] * (len(b) + 1)
    for x in a:
        cur = [0] * (len(b) + 1)
        for j, y in enumerate(b, 1):
            cur[j] = prev[j - 1] + 1 if x == y else max(prev[j], cur[j - 1])
        prev = cur
    return prev[-1]


def rouge_scores(pred: str, ref: str, use_stemmer: bool = True) -> Dict[str, Tuple[float, float, float]]:
    """{'rouge1'|'rouge2'|'rougeL': (precision, recall, fmeasure)}"""
    pt, rt = rouge_tokenize(pred, use_stemmer), rouge_tokenize(ref, use_stemmer)
    out = {}
    for n, key in ((1, "rouge1"), (2, "rouge2")):
        pc, rc = _ngrams(pt, n), _ngrams(rt, n)
        overlap = sum(min(c, rc[g]) for g, c in pc.items())
        out[key] = _f1(overlap, sum(pc.values()), sum(rc.values()))
    out["rougeL"] = _f1(_lcs(rt, pt), len(pt), len(rt))
    return out


def evaluate_rouge(pred: str, ref: str) -> Tuple[float, float, float]:
    s = rouge_scores(pred, ref)
    return s["rouge1"][2], s["rouge2"][2], s["rougeL"][2]


def mean_rouge(r1: float, r2: float, rl: float) -> float:
    return (r1 + r2 + rl) / 3.0


# ------------------------------------------------------------------------------ BLEU (13a)
_13A = [
    (re.compile(r"([\{-\~\[-\` -\&\(-\+\:-\@\/])"), r" \1 "),
    (re.compile(r"([^0-9])([\.,])"), r"\1 \2 "),
    (re.compile(r"([\.,])([^0-9])"), r" \1 \2"),
    (re.compile(r"([0-9])(-)"), r"\1 \2 "),
]


def tokenize_13a(line: str) -> List[str]:
    line = line.replace("<skipped>", "").replace("-\n", "").replace("\n", " ")
    if "&" in line:
        line = line.replace("&quot;", '"').replace("&amp;", "&").replace("&lt;", "<").replace("&gt;", ">")
    line = " " + line + " "
    for rx, rep in _13A:
        line = rx.sub(rep, line)
    return line.split()


def corpus_bleu(predictions: Sequence[str], references: Sequence[Sequence[str]], max_order: int = 4,
                smooth: bool = False) -> Dict[str, float]:
    matches = [0] * max_order
    possible = [0] * max_order
    ref_len = trans_len = 0
    for pred, refs in zip(predictions, references):
        pt = tokenize_13a(pred)
        rts = [tokenize_13a(r) for r in refs]
        ref_len += min(len(r) for r in rts)
        trans_len += len(pt)
        merged = Counter()
        for r in rts:
            for n in range(1, max_order + 1):
                merged |= _ngrams(r, n)
        for n in range(1, max_order + 1):
            pc = _ngrams(pt, n)
            matches[n - 1] += sum(min(c, merged[g]) for g, c in pc.items())
            possible[n - 1] += max(len(pt) - n + 1, 0)
    prec = []
    for i in range(max_order):
        if smooth:
            prec.append((matches[i] + 1.0) / (possible[i] + 1.0))
        else:
            prec.append(matches[i] / possible[i] if possible[i] > 0 else 0.0)
    geo = math.exp(sum(math.log(p) for p in prec) / max_order) if min(prec) > 0 else 0.0
    ratio = trans_len / ref_len if ref_len > 0 else 0.0
    bp = 1.0 if ratio > 1.0 else (math.exp(1 - 1.0 / ratio) if ratio > 0 else 0.0)
    return {"bleu": geo * bp, "precisions": prec, "brevity_penalty": bp, "length_ratio": ratio,
            "translation_length": trans_len, "reference_length": ref_len}


def evaluate_bleu(pred: str, ref: str) -> float:
    return corpus_bleu([pred], [[ref]])["bleu"]
