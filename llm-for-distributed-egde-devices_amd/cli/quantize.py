"""Write an edgellm INT8 checkpoint (quant/checkpoint.py format) for a model.

    python -m edgellm.cli.quantize --model llama-2-7b --quant w8a8_smoothquant --out /ckpt/llama-2-7b-w8a8
    python -m edgellm.cli.quantize --model /models/meta-llama_Llama-3.2-1B-Instruct --quant llm_int8 --out ...

The reference quantises at every load (``BitsAndBytesConfig(load_in_8bit=True)``,
Code/Quantised Models/models_quant_updated.py:30-38) and never stores INT8 weights.  Here the
model is loaded (a local HF checkpoint, else random-init weights of the named architecture),
quantised exactly as ``load_model(..., quant=...)`` does in memory (SmoothQuant: the same
calibration text, smoothing folded into the norms), and written once.  Every consumer then reads
the checkpoint directory as the model id — ``bench.py --checkpoint``, the evaluate / combine / serve
CLIs (``--models`` / YAML model paths), and each pipeline rank, which reads only its own stage
(``load_quantized(first=, last=)``) without building or calibrating the full bf16 model.
Tokenizer files of a source checkpoint directory are copied alongside.
"""
from __future__ import annotations

import argparse
import os
import shutil
import time
from typing import List, Optional

import torch

from ..models.hf import resolve_model_dir
from ..models.registry import load_model
from ..quant.checkpoint import save_quantized
from ..utils.log import get_logger

logger = get_logger("quantize")
_TOKENIZER_FILES = ("tokenizer.json", "tokenizer.model", "tokenizer_config.json", "special_tokens_map.json",
                    "vocab.json", "merges.txt", "vocab.txt")


def main(argv: Optional[List[str]] = None) -> str:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model", required=True, help="HF id / local checkpoint dir / architecture preset")
    ap.add_argument("--quant", default="w8a8_smoothquant", choices=["w8a8_smoothquant", "w8a8", "llm_int8"])
    ap.add_argument("--out", required=True, help="output directory")
    ap.add_argument("--precision", default="bf16", help="dtype of the non-quantised tensors (bf16 | fp16 | fp32)")
    ap.add_argument("--device", default=None, help="where to quantise (default cuda:0 when present, else cpu)")
    ap.add_argument("--base_model_path", default=None, help="directory holding downloaded checkpoints")
    a = ap.parse_args(argv)
    dev = torch.device(a.device or ("cuda:0" if torch.cuda.is_available() else "cpu"))
    t0 = time.perf_counter()
    model, _, source = load_model(a.model, a.precision, a.quant, dev, a.base_model_path)
    save_quantized(model, a.out, extra={"source": source, "model_id": a.model})
    src = resolve_model_dir(a.model, a.base_model_path)
    if src:
        for f in _TOKENIZER_FILES:
            if os.path.exists(os.path.join(src, f)):
                shutil.copy(os.path.join(src, f), os.path.join(a.out, f))
    size = os.path.getsize(os.path.join(a.out, "model.safetensors")) / 1e9
    logger.info(f"{a.model} ({source}) -> {a.out}: {a.quant}, {size:.2f} GB in {time.perf_counter() - t0:.1f} s")
    return a.out


if __name__ == "__main__":
    main()
