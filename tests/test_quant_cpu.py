import copy

import pytest
import torch

from edgellm.engine import KVCache
from edgellm.models import AttnCtx, build_model, tiny
from edgellm.quant import (LLMInt8Linear, W8A8Linear, collect_act_absmax, load_quantized, quantize_model,
                           save_quantized, smooth_model_, synthetic_calibration)


def _logits(model, ids):
    B, T = ids.shape
    kv = KVCache(model.cfg, B, T + 1, dtype=model.dtype)
    sp = torch.zeros(B, dtype=torch.int32)
    ctx = AttnCtx("prefill", B, T, sp, sp + T, T, kv, model.rope_table())
    return model(ids, ctx, logits="all").float()


@pytest.mark.parametrize("arch", ["llama", "llama2", "phi", "gpt_neox", "gpt2"])
def test_smoothing_fold_is_exact_in_fp32(arch):
    """Folding s into norms / v rows / up rows and W columns must not change the function."""
    cfg = tiny(arch)
    m = build_model(cfg, dtype=torch.float32, seed=3)
    ids = torch.randint(0, cfg.vocab_size, (2, 9))
    ref = _logits(m, ids)
    stats = collect_act_absmax(m, synthetic_calibration(cfg, 2, 16))
    factors = smooth_model_(m, stats, alpha=0.5)
    assert factors
    # apply the W side of the migration in fp32 (what the quantiser does before rounding)
    for j, layer in enumerate(m.layers):
        for mod, key in ((layer.attn.qkv, "attn.qkv"), (layer.attn.o, "attn.o"), (layer.mlp.up, "mlp.up"),
                         (layer.mlp.down, "mlp.down")):
            s = factors.get(f"layers.{j}.{key}")
            if s is not None:
                mod.weight.mul_(s[None, :])
    out = _logits(m, ids)
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-4), (out - ref).abs().max()


@pytest.mark.parametrize("mode", ["w8a8_smoothquant", "w8a8", "llm_int8", "cpu_dynamic"])
@pytest.mark.parametrize("arch", ["llama", "phi", "gpt_neox"])
def test_quantized_model_tracks_float(mode, arch):
    cfg = tiny(arch)
    m = build_model(cfg, dtype=torch.float32, seed=1)
    ids = torch.randint(0, cfg.vocab_size, (2, 12))
    ref = _logits(m, ids)
    q = quantize_model(copy.deepcopy(m).to(torch.bfloat16), mode)
    out = _logits(q, ids)
    rel = (out - ref).norm() / ref.norm()
    assert rel < 0.08, float(rel)
    # top-1 agreement on most positions
    agree = (out.argmax(-1) == ref.argmax(-1)).float().mean()
    assert agree > 0.7


def test_w8a8_linear_matches_dequant():
    torch.manual_seed(0)
    from edgellm.models.layers import Linear
    lin = Linear(96, 48, bias=True, dtype=torch.bfloat16)
    lin.weight.data.normal_(0, 0.05)
    lin.bias.data.normal_(0, 0.1)
    q = W8A8Linear.from_float(lin)
    x = torch.randn(5, 96).bfloat16()
    from edgellm import ops
    qx, sx = ops.quant_per_token(x)
    ref = (qx.float() * sx[:, None]) @ q.dequant_weight().t() + lin.bias.float()
    assert torch.allclose(q(x).float(), ref, atol=2e-2, rtol=1e-2)


def test_llm_int8_outlier_path():
    from edgellm.models.layers import Linear
    lin = Linear(64, 32, bias=False, dtype=torch.bfloat16)
    lin.weight.data.normal_(0, 0.05)
    q = LLMInt8Linear.from_float(lin, threshold=6.0)
    x = torch.randn(4, 64).bfloat16()
    x[:, 5] = 40.0                     # an outlier column goes through the bf16 path
    out = q(x).float()
    ref = x.float() @ lin.weight.float().t()
    assert ((out - ref).norm() / ref.norm()) < 0.02


@pytest.mark.parametrize("mode", ["w8a8_smoothquant", "llm_int8"])
def test_checkpoint_roundtrip(tmp_path, mode):
    cfg = tiny("llama")
    m = quantize_model(build_model(cfg, dtype=torch.bfloat16, seed=2), mode)
    ids = torch.randint(0, cfg.vocab_size, (1, 8))
    ref = _logits(m, ids)
    save_quantized(m, str(tmp_path))
    m2 = load_quantized(str(tmp_path))
    assert torch.equal(_logits(m2, ids), ref)
    # stage-sliced load gets the same layer weights
    st = load_quantized(str(tmp_path), first=1, last=2)
    assert st.layers[0].idx == 1 and isinstance(st.layers[0].attn.qkv, type(m.layers[1].attn.qkv))


def test_decode_rows_capability_table():
    """The 65-256 row decode kernels (ring2) take K % 128 == 0 (split-K: >= 4 stages of 128 k per
    slice at 65-128 rows): the Python gates (grouped attention output, split-K, fused GLU) must
    agree with the kernel table."""
    from edgellm import ops
    if not ops.available():
        pytest.skip("extension not built")
    assert all(ops.decode_rows_ok(M, K) for M in (1, 17, 64) for K in (64, 1000, 11008))
    assert ops.decode_rows_ok(128, 4096) and ops.decode_rows_ok(65, 4096) and ops.decode_rows_ok(100, 11008)
    assert not ops.decode_rows_ok(100, 1000) and not ops.decode_rows_ok(65, 4160)
    # 129-256 rows: the row-split ring2 kernels, any K % 128 == 0 with >= 8 stages
    assert ops.decode_rows_ok(129, 4096) and ops.decode_rows_ok(256, 11008, 4) and ops.decode_rows_ok(256, 1024)
    assert not ops.decode_rows_ok(257, 4096) and not ops.decode_rows_ok(200, 1000) and not ops.decode_rows_ok(200, 896)
    for K in (2048, 4096, 11008, 14336):                # o / down of 2048-hidden models, Llama-2-7B, Llama-3-8B
        assert ops.decode_rows_ok(128, K, 4)
    assert not ops.decode_rows_ok(128, 1024, 4)         # 8 stages over 4 slices: < 4 per slice
    lin = W8A8Linear(11008, 4096, bias=False)
    assert lin.group_scales_ok(128) and lin.group_scales_ok(64)
    up = W8A8Linear(4096, 22016, bias=False)
    assert up.glu_rows_ok(128) and W8A8Linear(2048, 11008, bias=False).glu_rows_ok(100)
    assert not W8A8Linear(1000, 11008, bias=False).glu_rows_ok(100)


@pytest.mark.parametrize("bounds", [[0, 3, 8], [0, 5, 11, 16]])
def test_smoothquant_stage_p2p_equals_full_model_calibration(bounds):
    """Per-stage SmoothQuant (each stage calibrated on the activations the previous stage sends
    it, no rank building the full model) gives the same int8 weights, scales and folded norms as
    calibrating the full model and cutting the stage — fp32, whole-layer and half-layer bounds."""
    from edgellm.models.decoder import global_named_parameters
    from edgellm.quant.smoothquant import smoothquant_stage, smoothquant_stage_p2p, synthetic_calibration
    cfg = tiny("llama", num_layers=8)
    calib = synthetic_calibration(cfg, n=2, T=16, seed=3)
    full = build_model(cfg, dtype=torch.float32, seed=7)
    units = len(bounds) == 4 or bounds[-1] == 16
    box = {}

    def recv(shape, dtype):
        t = box.pop("h")
        assert tuple(t.shape) == tuple(shape) and t.dtype == dtype
        return t

    def send(t):
        box["h"] = t

    for s in range(len(bounds) - 1):
        a, b = bounds[s], bounds[s + 1]
        kw = dict(units=(a, b)) if units else dict(first=a, last=b)
        ref = smoothquant_stage(copy.deepcopy(full), a, b, calib, units=(a, b) if units else None)
        got = smoothquant_stage_p2p(cfg, calib, recv, send, dtype=torch.float32, seed=7, **kw)
        rb = dict(global_named_parameters(ref))
        gb = dict(global_named_parameters(got))
        assert rb.keys() == gb.keys()
        for k in rb:
            assert torch.equal(rb[k], gb[k]), k
        rbuf = dict(ref.named_buffers())
        for k, v in got.named_buffers():
            assert torch.equal(v, rbuf[k]), k
    assert not box, "the last stage sends nothing"
