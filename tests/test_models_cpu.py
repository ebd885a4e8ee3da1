"""Model-zoo parity against Hugging Face transformers (the reference's runtime), on CPU.

Each family is built from a tiny random-init HF config, converted with edgellm.models.hf and
compared logit-by-logit (prefill) and through a prefill + decode split (KV cache path).
"""
import pytest
import torch

from edgellm.engine import KVCache
from edgellm.models import AttnCtx, tiny
from edgellm.models.configs import from_hf_config
from edgellm.models.hf import from_hf_module

transformers = pytest.importorskip("transformers")


def _hf_model(arch):
    T = transformers
    if arch == "llama":
        c = T.LlamaConfig(vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                          num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256,
                          rope_theta=500000.0, tie_word_embeddings=True,
                          rope_scaling={"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                                        "high_freq_factor": 4.0, "original_max_position_embeddings": 64})
        return T.LlamaForCausalLM(c)
    if arch == "gpt_neox":
        c = T.GPTNeoXConfig(vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                            num_attention_heads=2, rotary_pct=0.25, max_position_embeddings=256)
        return T.GPTNeoXForCausalLM(c)
    if arch == "phi":
        c = T.PhiConfig(vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                        num_attention_heads=2, partial_rotary_factor=0.5, max_position_embeddings=256)
        return T.PhiForCausalLM(c)
    if arch == "gpt2":
        c = T.GPT2Config(vocab_size=300, n_embd=64, n_layer=2, n_head=2, n_positions=256)
        return T.GPT2LMHeadModel(c)
    raise ValueError(arch)


def _run(model, ids, kv, start, mode):
    B, T = ids.shape
    sp = torch.full((B,), start, dtype=torch.int32)
    ctx = AttnCtx(mode, B, T, sp, sp + T, start + T, kv, model.rope_table())
    return model(ids, ctx, logits="all").float()


@pytest.mark.parametrize("arch", ["llama", "gpt_neox", "phi", "gpt2"])
def test_family_matches_hf(arch):
    torch.manual_seed(0)
    hf = _hf_model(arch).eval().float()
    for p in hf.parameters():  # larger weights so differences are visible
        p.data.normal_(0, 0.1)
    cfg = from_hf_config(hf.config.to_dict())
    ours = from_hf_module(hf, cfg, dtype=torch.float32)
    ids = torch.randint(0, 300, (2, 40))
    with torch.no_grad():
        ref = hf(ids).logits.float()
    kv = KVCache(cfg, 2, 64, dtype=torch.float32)
    out = _run(ours, ids, kv, 0, "prefill").view(2, 40, -1)
    assert torch.allclose(out, ref, atol=2e-4, rtol=1e-3), (out - ref).abs().max()
    # prefill 33 tokens, then decode the remaining 7 one by one through the KV cache
    kv = KVCache(cfg, 2, 64, dtype=torch.float32)
    _run(ours, ids[:, :33], kv, 0, "prefill")
    for t in range(33, 40):
        step = _run(ours, ids[:, t:t + 1], kv, t, "decode")
        assert torch.allclose(step.view(2, -1), ref[:, t], atol=2e-4, rtol=1e-3)


def test_bf16_model_runs_and_presets():
    from edgellm.models import PRESETS, build_model
    for name in ("llama-2-7b", "llama-3-8b", "llama-3.2-1b", "phi-2", "pythia-1b", "gpt2"):
        assert PRESETS[name].num_params() > 1e8
    assert abs(PRESETS["llama-2-7b"].num_params() / 1e9 - 6.74) < 0.05
    cfg = tiny("llama")
    m = build_model(cfg, dtype=torch.bfloat16)
    kv = KVCache(cfg, 1, 32, dtype=torch.bfloat16)
    out = _run(m, torch.randint(0, cfg.vocab_size, (1, 5)), kv, 0, "prefill")
    assert out.shape == (5, cfg.vocab_size) and torch.isfinite(out).all()


def test_stage_split_weights_identical():
    from edgellm.models import build_model, global_named_parameters
    cfg = tiny("llama", num_layers=4)
    full = dict(global_named_parameters(build_model(cfg, dtype=torch.float32)))
    for a, b in ((0, 2), (2, 4), (1, 3)):
        st = build_model(cfg, dtype=torch.float32, first=a, last=b)
        for n, p in global_named_parameters(st):
            ref = full["embed"] if (n == "lm_head.weight" and cfg.tie_word_embeddings) else full[n]
            assert torch.equal(p, ref), n


@pytest.mark.parametrize("arch", ["llama", "llama2", "gpt_neox", "phi", "gpt2"])
def test_hf_export_roundtrip_loads_in_transformers(arch, tmp_path):
    """save_hf_model writes a save_pretrained-format dir: edgellm reloads it bit-exactly and
    transformers' own loader produces the same logits (the exporter is the inverse converter)."""
    from edgellm.models import build_model, global_named_parameters
    from edgellm.models.hf import load_hf_model, save_hf_model
    cfg = tiny(arch)
    m = build_model(cfg, dtype=torch.float32, seed=5)
    save_hf_model(m, str(tmp_path / "ck"))
    back = load_hf_model(str(tmp_path / "ck"), dtype=torch.float32)
    a, b = dict(global_named_parameters(m)), dict(global_named_parameters(back))
    assert a.keys() == b.keys() and all(torch.equal(a[k], b[k]) for k in a)
    hf = transformers.AutoModelForCausalLM.from_pretrained(str(tmp_path / "ck"), torch_dtype=torch.float32).eval()
    ids = torch.randint(0, cfg.vocab_size, (2, 12))
    with torch.no_grad():
        ref = hf(ids).logits.float()
    kv = KVCache(cfg, 2, 32, dtype=torch.float32)
    out = _run(m, ids, kv, 0, "prefill").view(2, 12, -1)
    assert torch.allclose(out, ref, atol=2e-4, rtol=1e-3), (out - ref).abs().max()


def test_fetch_random_init_layout(tmp_path):
    """cli.fetch writes the reference downloader's BASE_DIR/<org>_<name> layout (download.py:22)
    offline, and the registry resolves the model from it."""
    from edgellm.cli.fetch import fetch_dataset, fetch_model
    from edgellm.models.registry import load_model
    base = str(tmp_path)
    d = fetch_model("acme/tiny-llama", base, random_init=True, cfg_override=tiny("llama"))
    assert d == str(tmp_path / "acme_tiny-llama") and (tmp_path / "acme_tiny-llama" / "RANDOM_INIT").exists()
    assert fetch_model("acme/tiny-llama", base) == d           # present: kept
    model, tok, src = load_model("acme/tiny-llama", "fp32", "none", "cpu", base_dir=base)
    assert model.cfg.hidden_size == tiny("llama").hidden_size and "acme_tiny-llama" in src
    csv_path = fetch_dataset("sentence-transformers/natural-questions", "train[:3]", base)
    assert open(csv_path).read().splitlines()[0] == "query,answer"
