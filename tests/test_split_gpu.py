"""SplitLM (parallel/split.py, the reference's ``device_map="auto"`` layer split) on the GPU.

The box has one MI355X, so the cross-device cases are a 2-stage split with both stages on cuda:0
(per-stage KV caches and the stage hop, every custom kernel launched through the bindings'
device guard) and a CPU -> cuda:0 split (a real device change between stages: stage 0 runs the
fp32 reference ops on the host, stage 1 the HIP kernels).  Logits and greedy tokens are compared
with the unsplit model.
"""
import copy

import pytest
import torch

from edgellm.engine import Generator, SamplingParams
from edgellm.models import build_model, tiny
from edgellm.parallel.split import SplitLM
from edgellm.quant import quantize_model

pytestmark = pytest.mark.gpu


def _model(dev, quant):
    cfg = tiny("llama", hidden_size=256, num_heads=4, num_kv_heads=2, intermediate_size=512, num_layers=4)
    m = build_model(cfg, device=dev, seed=3)
    return quantize_model(m, quant) if quant != "none" else m


def _greedy(model, prompts, n=12):
    gen = Generator(model, max_batch=len(prompts), max_seq=64)
    res = gen.generate(prompts, SamplingParams(max_new_tokens=n, do_sample=False), seed=0)
    return res.tokens


@pytest.mark.parametrize("quant", ["none", "w8a8_smoothquant"])
def test_split_same_device_matches_unsplit(cuda, quant):
    base = _model(cuda, quant)
    split = SplitLM(copy.deepcopy(base), [cuda, cuda], bounds=[0, 2, 4])
    prompts = [[5, 9, 13, 2, 7, 1, 8, 3]] * 2 + [[4, 4, 11, 6, 2, 9, 1, 5]]
    assert _greedy(split, prompts) == _greedy(base, prompts)


@pytest.mark.parametrize("quant", ["none", "w8a8_smoothquant"])
def test_split_cpu_then_gpu(cuda, quant):
    """Stage 0 on the host, stage 1 + head on cuda:0: logits of one prefill agree with the unsplit
    GPU model to the HIP-vs-reference tolerance."""
    from edgellm.models import AttnCtx
    base = _model(cuda, quant)
    split = SplitLM(copy.deepcopy(base), [torch.device("cpu"), cuda], bounds=[0, 2, 4])
    ids = torch.tensor([[5, 9, 13, 2, 7, 1, 8, 3]])
    outs = []
    for m, dev in ((base, cuda), (split, torch.device("cpu"))):
        kv = m.make_kv(1, 32) if hasattr(m, "make_kv") else \
            __import__("edgellm.engine", fromlist=["KVCache"]).KVCache(m.cfg, 1, 32, dtype=m.dtype, device=cuda)
        sp = torch.zeros(1, dtype=torch.int32, device=dev)
        ctx = AttnCtx("prefill", 1, 8, sp, sp + 8, 8, kv.rows(0, 1), m.rope_table(dev))
        with torch.no_grad():
            outs.append(m(ids.to(dev), ctx).float().cpu())
    a, b = outs
    rel = ((a - b).norm() / b.norm()).item()
    assert rel < (2e-2 if quant == "none" else 6e-2), rel
