"""QA datasets with the reference's schema: rows of {"query", "answer"}.

Sources, in order: a CSV path (Code/Dataset/natural_questions_1000.csv format, read as in
try.py:292), an HF ``datasets`` name available in the local cache (load_dataset(name, split,
cache_dir) as in combine_model_fp_updated.py:171 — offline only), else the bundled 10-row
sample of that CSV (``nq_sample.csv``, passages truncated) so every entry point runs.
Split strings "train[:1000]" / "train[10:20]" are honoured for every source.
"""
from __future__ import annotations

import csv
import os
import re
from typing import Dict, List, Optional

HERE = os.path.dirname(os.path.abspath(__file__))
SAMPLE_CSV = os.path.join(HERE, "nq_sample.csv")


def _slice(split: Optional[str]):
    if not split:
        return slice(None)
    m = re.search(r"\[(\-?\d*):(\-?\d*)\]", split)
    if not m:
        return slice(None)
    a, b = m.group(1), m.group(2)
    return slice(int(a) if a else None, int(b) if b else None)


def read_csv(path: str) -> List[Dict[str, str]]:
    with open(path, newline="", encoding="utf-8") as f:
        return [{"query": r["query"], "answer": r["answer"]} for r in csv.DictReader(f)]


def load_qa(name: Optional[str] = None, split: Optional[str] = None, path: Optional[str] = None,
            limit: Optional[int] = None) -> List[Dict[str, str]]:
    rows = None
    for cand in (path, name):
        if cand and os.path.isfile(cand) and cand.endswith(".csv"):
            rows = read_csv(cand)
            break
    if rows is None and name and not os.path.isfile(name):
        try:
            os.environ.setdefault("HF_DATASETS_OFFLINE", "1")
            import datasets
            ds = datasets.load_dataset(name, split=(split or "train").split("[")[0], cache_dir=path)
            rows = [{"query": r["query"], "answer": r["answer"]} for r in ds]
        except Exception:
            rows = None
    if rows is None:
        rows = read_csv(SAMPLE_CSV)
    rows = rows[_slice(split)]
    return rows[:limit] if limit else rows
