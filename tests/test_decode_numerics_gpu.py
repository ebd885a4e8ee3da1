"""Model-level DECODE numerics: the fused HIP decode step (fused RoPE + KV append + attention,
split-K o / down, quantising GLU, 65-128-row kernels, bf16 GEMVs) against the fp32 reference ops
(``EDGELLM_REF_ON_GPU`` routing, same weights, same KV cache), at Llama-2-7B layer shapes.

Bounded on the relative error of the decode-step logits, at micro-batch
sizes that select every decode kernel family: 1 (GEMV), 16 / 64 (grouped-scale GEMVs), 128 (the
LDS-staged / ring kernels), 200 / 256 (the row-split ring2 kernels of one 256-row micro-batch).
"""
import pytest
import torch

from edgellm import ops
from edgellm.engine import KVCache
from edgellm.models import AttnCtx, build_model, get_config
from edgellm.quant import quantize_model

pytestmark = pytest.mark.gpu

_MODELS = {}


def _model(cuda, quant):
    key = quant
    if key not in _MODELS:
        cfg = get_config("llama-2-7b").replace(num_layers=2)
        m = build_model(cfg, device=cuda, seed=11)
        if quant != "none":
            m = quantize_model(m, quant)
        _MODELS[key] = m
    return _MODELS[key]


def _decode_logits(model, kv, tok, pos, dev):
    B = tok.shape[0]
    seq = pos + 1
    ctx = AttnCtx("decode", B, 1, pos, seq, int(seq.max().item()), kv.rows(0, B), model.rope_table(dev))
    return model(tok.view(B, 1), ctx).float()


@pytest.mark.parametrize("B", [1, 16, 64, 128, 200, 256])
@pytest.mark.parametrize("quant", ["none", "w8a8_smoothquant"])
def test_decode_step_logits_match_fp32_reference(cuda, B, quant, monkeypatch):
    model = _model(cuda, quant)
    cfg = model.cfg
    T = 24
    g = torch.Generator().manual_seed(B)
    ids = torch.randint(0, cfg.vocab_size, (B, T), generator=g).to(cuda)
    kv = KVCache(cfg, B, T + 8, dtype=model.dtype, device=cuda)
    sp = torch.zeros(B, dtype=torch.int32, device=cuda)
    with torch.no_grad():
        model(ids, AttnCtx("prefill", B, T, sp, sp + T, T, kv.rows(0, B), model.rope_table(cuda)), logits="last")
        k0, v0 = kv.k.clone(), kv.v.clone()
        tok = torch.randint(0, cfg.vocab_size, (B,), generator=g).to(cuda)
        pos = torch.full((B,), T, dtype=torch.int32, device=cuda)
        hip = _decode_logits(model, kv, tok, pos, cuda)
        k_hip = kv.k[:, :, :, T].clone()
        kv.k.copy_(k0)
        kv.v.copy_(v0)
        monkeypatch.setattr(ops, "_REF_ON_GPU", True)
        ref = _decode_logits(model, kv, tok, pos, cuda)
        monkeypatch.setattr(ops, "_REF_ON_GPU", False)
    assert torch.isfinite(hip).all()
    rel = ((hip - ref).norm(dim=-1) / ref.norm(dim=-1))           # per row: a broken row block shows
    tol = 2e-2 if quant == "none" else 4e-2
    assert rel.max().item() < tol, (rel.max().item(), rel.argmax().item())
    # the fused append wrote the same rotated key rows the reference wrote (relative, per layer)
    for li in range(cfg.num_layers):
        a, b = k_hip[li].float(), kv.k[li, :, :, T].float()
        assert ((a - b).norm() / b.norm()).item() < 2e-2, li
