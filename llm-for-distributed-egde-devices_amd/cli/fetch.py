"""Provision models, embedder and dataset into a BASE_DIR (reference: Code/C-DAC Server/download.py,
Code/others/download(1).py).

Same on-disk layout as the reference downloader, so every loader here (and the reference's own
scripts) finds the assets:

    BASE_DIR/<org>_<name>/            config.json + *.safetensors (+ tokenizer files)
    BASE_DIR/natural_questions_1000.csv   query,answer rows of the dataset split

Sources, in order, for each model: an existing ``BASE_DIR/<org>_<name>`` (kept), the local
Hugging Face cache (``local_files_only``), a download (only with ``--online``), or — with
``--random-init`` — a random-init checkpoint of the named architecture written in HF format
(benchmarks and tests; there is no network in CI).  The BLEU/BERTScore metric code the
reference pre-fetches is built into ``edgellm.eval``, so nothing is fetched for it.

    python -m edgellm.cli.fetch --base_dir /data/models --random-init
"""
from __future__ import annotations

import argparse
import csv
import os
from typing import List, Optional

from ..utils.log import get_logger

log = get_logger("fetch")

DEFAULT_MODELS = ["microsoft/phi-2", "EleutherAI/pythia-1b", "meta-llama/Llama-3.2-1B-Instruct"]
DEFAULT_EMBEDDER = "sentence-transformers/all-MiniLM-L6-v2"
DEFAULT_DATASET = "sentence-transformers/natural-questions"

_PRESET_OF = {"microsoft/phi-2": "phi-2", "EleutherAI/pythia-1b": "pythia-1b",
              "meta-llama/Llama-3.2-1B-Instruct": "llama-3.2-1b", "meta-llama/Llama-2-7b-hf": "llama-2-7b",
              "meta-llama/Meta-Llama-3-8B": "llama-3-8b", "gpt2": "gpt2", "openai-community/gpt2": "gpt2",
              DEFAULT_EMBEDDER: "minilm-l6"}


def target_dir(base_dir: str, name: str) -> str:
    return os.path.join(base_dir, name.replace("/", "_"))        # download.py:22 layout


def _from_hf(name: str, dst: str, online: bool) -> bool:
    """Copy a checkpoint from the HF cache (or the hub when ``online``) with save_pretrained."""
    try:
        import transformers as T
        kw = dict(local_files_only=not online)
        tok = T.AutoTokenizer.from_pretrained(name, **kw)
        model = T.AutoModelForCausalLM.from_pretrained(name, torch_dtype="auto", **kw)
    except Exception as e:  # not cached / offline
        log.info(f"{name}: not available from the HF cache ({type(e).__name__})")
        return False
    tok.save_pretrained(dst)
    model.save_pretrained(dst, safe_serialization=True)
    return True


def fetch_model(name: str, base_dir: str, online: bool = False, random_init: bool = False,
                dtype: str = "bfloat16", seed: int = 0, cfg_override=None) -> Optional[str]:
    dst = target_dir(base_dir, name)
    if os.path.isfile(os.path.join(dst, "config.json")):
        log.info(f"{name}: present at {dst}")
        return dst
    print(f"Downloading: {name}")
    if _from_hf(name, dst, online):
        return dst
    if not random_init:
        log.warning(f"{name}: skipped (offline and not cached; pass --random-init to write a random-init checkpoint)")
        return None
    import torch
    from ..models import build_model
    from ..models.configs import get_config
    from ..models.hf import save_hf_model
    cfg = cfg_override or get_config(_PRESET_OF.get(name, name))
    if cfg.arch == "bert":
        log.warning(f"{name}: random-init export is not supported for encoders; the embedder falls back "
                    "to random init at load time")
        return None
    model = build_model(cfg, dtype=getattr(torch, dtype), device="cpu", seed=seed)
    save_hf_model(model, dst)
    with open(os.path.join(dst, "RANDOM_INIT"), "w") as f:
        f.write(f"random-init weights of the {cfg.name or cfg.arch} architecture (seed {seed}); not a trained model\n")
    log.info(f"{name}: wrote random-init checkpoint to {dst}")
    return dst


def fetch_dataset(name: str, split: str, base_dir: str, path: Optional[str] = None) -> str:
    from ..data import load_qa
    print(f"Downloading dataset: {name}")
    rows = load_qa(name, split, path)
    out = os.path.join(base_dir, "natural_questions_1000.csv")
    with open(out, "w", newline="", encoding="utf-8") as f:
        w = csv.DictWriter(f, fieldnames=["query", "answer"])
        w.writeheader()
        w.writerows(rows)
    log.info(f"dataset: {len(rows)} rows -> {out}")
    return out


def main(argv: Optional[List[str]] = None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--base_dir", default=os.environ.get("EDGELLM_MODELS", "models"))
    ap.add_argument("--models", nargs="*", default=DEFAULT_MODELS)
    ap.add_argument("--embedder", default=DEFAULT_EMBEDDER)
    ap.add_argument("--dataset", default=DEFAULT_DATASET)
    ap.add_argument("--split", default="train[:1000]")
    ap.add_argument("--dataset_path", default=None, help="CSV to export instead of the HF dataset")
    ap.add_argument("--online", action="store_true", help="allow hub downloads (off: cache only)")
    ap.add_argument("--random-init", action="store_true", help="write random-init checkpoints for missing models")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    os.makedirs(a.base_dir, exist_ok=True)
    got = {m: fetch_model(m, a.base_dir, a.online, a.random_init, seed=a.seed) for m in a.models}
    if a.embedder:
        print(f"Downloading embedder: {a.embedder}")
        got[a.embedder] = target_dir(a.base_dir, a.embedder) if _from_hf_encoder(a.embedder, a.base_dir, a.online) \
            else None
    fetch_dataset(a.dataset, a.split, a.base_dir, a.dataset_path)
    print(f"\nAssets in {a.base_dir}: " + ", ".join(f"{k} -> {'ok' if v else 'missing'}" for k, v in got.items()))
    return got


def _from_hf_encoder(name: str, base_dir: str, online: bool) -> bool:
    dst = target_dir(base_dir, name)
    if os.path.isfile(os.path.join(dst, "config.json")):
        return True
    try:
        import transformers as T
        kw = dict(local_files_only=not online)
        T.AutoTokenizer.from_pretrained(name, **kw).save_pretrained(dst)
        T.AutoModel.from_pretrained(name, **kw).save_pretrained(dst, safe_serialization=True)
        return True
    except Exception as e:
        log.info(f"{name}: not available ({type(e).__name__}); the embedder will use random init")
        return False


if __name__ == "__main__":
    main()
