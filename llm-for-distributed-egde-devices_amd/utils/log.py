"""Logging with the reference's line format.

The reference logs every result line as ``"%(asctime)s - %(levelname)s - %(message)s"``
to stdout (Code/Base Models/combine_model_fp_updated.py:22-29,
Code/Base Models/Llama_bf16_updated.py:17).  ``get_logger`` reproduces that format so
result logs stay diff-able against the reference's pasted log (XLSX Results!E41:E49).
"""
import logging
import sys

LOG_FORMAT = "%(asctime)s - %(levelname)s - %(message)s"

_configured = False


def get_logger(name: str = "edgellm", level: int = logging.INFO) -> logging.Logger:
    global _configured
    if not _configured:
        handler = logging.StreamHandler(sys.stdout)
        handler.setFormatter(logging.Formatter(LOG_FORMAT))
        root = logging.getLogger("edgellm")
        root.addHandler(handler)
        root.setLevel(level)
        root.propagate = False
        _configured = True
    if not name.startswith("edgellm"):
        name = "edgellm." + name
    return logging.getLogger(name)


def format_final_report(means: dict) -> list:
    """The nine final lines of the ensemble scripts, same labels and widths
    (combine_model_fp_updated.py:223-232)."""
    r1, r2, rl = means["rouge1"], means["rouge2"], means["rougeL"]
    return [
        "\nFinal Evaluation:",
        f"ROUGE-1        → {r1:.4f}",
        f"ROUGE-2        → {r2:.4f}",
        f"ROUGE-L        → {rl:.4f}",
        f"Mean ROUGE     → {(r1 + r2 + rl) / 3.0:.4f}",
        f"BERTScore      → {means['bertscore']:.4f}",
        f"BLEU           → {means['bleu']:.4f}",
        f"Cosine Sim     → {means['cosine']:.4f}",
        f"Confidence     → {means['confidence']:.4f}",
        f"Tokens/Sec     → {means['tps']:.2f}",
    ]


def format_efficiency_report(means: dict) -> list:
    """Efficiency lines in the layout of the paper's Table 3 (memory, time, tokens/sec), after
    the reference's nine lines: time = whole-loop wall per sample (tqdm s/it), metrics included."""
    t = means.get("total_time_s", 0.0)
    h, rem = divmod(int(round(t)), 3600)
    m, s = divmod(rem, 60)
    return [
        f"Time Taken     → {h}:{m:02d}:{s:02d} ({means.get('time_per_sample_s', 0.0):.2f} s/it)",
        f"Memory (GB)    → {means.get('peak_mem_gb', 0.0):.2f}",
        f"Agg. Tok/Sec   → {means.get('agg_tokens_per_s', 0.0):.2f}",
    ]


def format_single_model_report(means: dict) -> list:
    """Final lines of the single-model evaluators (Llama_bf16_updated.py:126-134)."""
    r1, r2, rl = means["rouge1"], means["rouge2"], means["rougeL"]
    return [
        f"ROUGE-1         → {r1:.4f}",
        f"ROUGE-2         → {r2:.4f}",
        f"ROUGE-L         → {rl:.4f}",
        f"BERTScore       → {means['bertscore']:.4f}",
        f"BLEU Score      → {means['bleu']:.4f}",
        f"Confidence Score→ {means['confidence']:.4f}",
        f"Similarity Score→ {means['cosine']:.4f}",
        f"Tokens/sec      → {means['tps']:.4f}",
        f" Mean ROUGE     → {(r1 + r2 + rl) / 3.0:.4f}",
    ]
