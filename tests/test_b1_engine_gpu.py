"""Batch-1 persistent decode engine (ops/csrc/b1_engine.hip) on the GPU.

* Stage by stage against a plain fp32 torch emulation of the same W8A8 math, computed from the
  canonical int8 weights and fed, stage by stage, the engine's own previous output (its granule
  buffers keep the last launch's values): qkv, the appended K / V rows, the int8 attention output and
  its per-64 scales, h2 = x + o, the SwiGLU output h, the layer output.
* End to end against the unquantised bf16 model: the engine's logits must be as close to it as the
  launch-per-op W8A8 path's (the two W8A8 paths round at different points: the launch path sums the
  o / down split-K slices of bf16-rounded partials and quantises the fp32 SwiGLU output, the engine
  accumulates o / down in fp32 and rounds h to bf16 as HF's bf16 MLP does).
* Through ``Generator``: HIP graph capture and replay of the one-launch decode step.
Shapes: Llama-2-7B (MHA, F 11008: uneven gate_up units), Llama-3-8B (GQA 32 / 8, F 14336),
Llama-3.2-1B (head_dim 64, H 2048: half the CUs own no o / down unit), cut to a few layers."""
import dataclasses
import struct

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [("llama-2-7b", 2, 100), ("llama-3-8b", 2, 37), ("llama-3.2-1b", 2, 200)]


def _cfg(name, layers):
    from edgellm.models import get_config
    return dataclasses.replace(get_config(name), num_layers=layers, vocab_size=4096, max_position_embeddings=1024)


def _model(cfg, dev, quant=True):
    from edgellm.models import build_model
    from edgellm.quant import quantize_model
    m = build_model(cfg, device=dev, seed=3)
    return quantize_model(m, "w8a8_smoothquant") if quant else m


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _bf(x):
    return x.to(torch.bfloat16).float()


def _unpack3(buf, counts):
    """Granule blocks [G, gpc] of 3 bf16 (+ 16-bit tag) -> the concatenated values."""
    b = buf.cpu()
    lo = (b & 0xFFFF).to(torch.int32)
    mid = ((b >> 16) & 0xFFFF).to(torch.int32)
    hi = ((b >> 32) & 0xFFFF).to(torch.int32)
    vals = torch.stack([lo, mid, hi], -1).reshape(b.shape[0], -1)        # [G, 3 gpc]
    f = (vals << 16).view(torch.float32)
    return torch.cat([f[c, :n] for c, n in enumerate(counts)])


def _unpack_att(ga):
    """[Hq, NGR, 12] granules -> (int8 values [Hq NGR, 64], scales [Hq NGR])."""
    g = ga.reshape(-1, 12).cpu()
    q = torch.zeros(g.shape[0], 64)
    s = torch.zeros(g.shape[0])
    for i in range(g.shape[0]):
        byts = []
        for j in range(11):
            v = int(g[i, j]) & ((1 << 48) - 1)
            byts += [(v >> (8 * k)) & 0xFF for k in range(6 if j < 10 else 4)]
        q[i] = torch.tensor([x - 256 if x > 127 else x for x in byts], dtype=torch.float32)
        s[i] = struct.unpack("<f", struct.pack("<I", int(g[i, 11]) & 0xFFFFFFFF))[0]
    return q, s


def _qgroup(x):
    x = x.view(-1, 64)
    s = x.abs().amax(1).clamp_min(1e-8) / 127
    return torch.round(x / s[:, None]).clamp(-127, 127), s


def _setup(name, layers, plen, dev, max_seq=512):
    from edgellm.engine.generate import Generator
    cfg = _cfg(name, layers)
    model = _model(cfg, dev)
    gen = Generator(model, max_batch=1, max_seq=max_seq, use_graphs=False)
    g = torch.Generator().manual_seed(1)
    gen.prefill(torch.randint(0, cfg.vocab_size, (1, plen), generator=g).to(dev))
    return cfg, model, gen.kv, g


@pytest.mark.parametrize("name,layers,plen", SHAPES)
def test_b1_engine_stages_match_fp32_emulation(cuda, name, layers, plen):
    from edgellm.engine import b1_engine
    dev = torch.device("cuda", 0)
    cfg, model, kv, g = _setup(name, layers, plen, dev)
    k0, v0 = kv.k.clone(), kv.v.clone()
    tok = torch.randint(0, cfg.vocab_size, (1,), generator=g).to(dev)
    sp = torch.full((1,), plen, dtype=torch.int32, device=dev)
    eng = b1_engine.engine_for(model, kv)
    assert eng is not None
    x0 = model.embed[tok].contiguous()
    xout = eng.run(x0, sp).float().reshape(-1).clone()
    torch.cuda.synchronize()
    eng.check()
    w = eng.w
    G, H, F, Hq, Hkv, HD = w.G, w.H, w.F, w.Hq, w.Hkv, w.HD
    split = b1_engine.unit_split
    cnt_h = [16 * int(n) for n in split(H // 16, G).diff()]
    cnt_q = [16 * int(n) for n in split(w.NQ // 16, G).diff()]
    cnt_f = [8 * int(n) for n in split(F // 8, G).diff()]
    rope = model.rope_table(dev)[plen]
    c_, s_ = rope[:, 0], rope[:, 1]
    rot = lambda t: torch.cat([t[:, :HD // 2] * c_ - t[:, HD // 2:] * s_, t[:, HD // 2:] * c_ + t[:, :HD // 2] * s_], 1)  # noqa
    x = x0.float().reshape(-1)
    for l, layer in enumerate(model.layers):
        (wq, sq, _), (wo, so, _), (wu, su, _), (wd, sd, _) = (
            m.canonical() for m in (layer.attn.qkv, layer.attn.o, layer.mlp.up, layer.mlp.down))
        # qkv: RMSNorm -> per-token int8 -> int32 dot -> scales -> bf16
        y = x * layer.norm1.weight.float() * torch.rsqrt(x.pow(2).mean() + w.eps)
        sa = y.abs().max().clamp_min(1e-8) / 127
        qkv = _bf((torch.round(y / sa).clamp(-127, 127) @ wq.float().t()) * sa * sq.float())
        e_qkv = _unpack3(eng.gq[l], cnt_q).to(dev)
        assert _rel(e_qkv, qkv) < 5e-3, (l, "qkv", _rel(e_qkv, qkv))
        q = e_qkv[:Hq * HD].view(Hq, HD)
        k = e_qkv[Hq * HD:(Hq + Hkv) * HD].view(Hkv, HD)
        v = e_qkv[(Hq + Hkv) * HD:].view(Hkv, HD)
        qr, kr = _bf(rot(q)), _bf(rot(k))
        assert _rel(kv.k[l, 0, :, plen].float(), kr) < 5e-3 and _rel(kv.v[l, 0, :, plen].float(), v) < 5e-3
        assert torch.equal(kv.k[l, 0, :, :plen], k0[l, 0, :, :plen])
        kc, vc = k0[l, 0].float(), v0[l, 0].float()
        kc[:, plen], vc[:, plen] = kr, v
        grp = Hq // Hkv
        att = _bf(torch.cat([torch.softmax((kc[h // grp, :plen + 1] @ qr[h]) * w.scale, 0) @ vc[h // grp, :plen + 1]
                             for h in range(Hq)]))
        aq, asc = _qgroup(att)
        e_aq, e_as = _unpack_att(eng.ga[l])
        assert _rel(e_aq * e_as[:, None], (aq * asc[:, None]).cpu()) < 5e-3, (l, "attention")
        # o: grouped scales, fp32 accumulate, + residual -> bf16
        e_aq, e_as = e_aq.to(dev), e_as.to(dev)
        o = (torch.einsum("ngk,gk->ng", wo.float().view(H, -1, 64), e_aq) * e_as[None]).sum(1) * so.float()
        h2 = _bf(o + x)
        e_h2 = _unpack3(eng.gr[l], cnt_h).to(dev)
        assert _rel(e_h2, h2) < 2e-3, (l, "h2", _rel(e_h2, h2))
        # gate_up + SwiGLU (bf16 g, u, h)
        y = e_h2 * layer.norm2.weight.float() * torch.rsqrt(e_h2.pow(2).mean() + w.eps)
        sa = y.abs().max().clamp_min(1e-8) / 127
        gu = (torch.round(y / sa).clamp(-127, 127) @ wu.float().t()) * sa * su.float()
        gg, uu = _bf(gu[:F]), _bf(gu[F:])
        hh = _bf(gg / (1 + torch.exp(-gg)) * uu)
        e_h = _unpack3(eng.gh[l], cnt_f).to(dev)
        assert _rel(e_h, hh) < 5e-3, (l, "h", _rel(e_h, hh))
        # down: per-64 int8 of h, grouped scales, + h2 -> bf16
        hq, hs = _qgroup(e_h)
        dn = (torch.einsum("ngk,gk->ng", wd.float().view(H, -1, 64), hq) * hs[None]).sum(1) * sd.float()
        x = _bf(dn + e_h2)
    assert _rel(xout, x) < 2e-3, _rel(xout, x)


@pytest.mark.parametrize("name,layers,plen", SHAPES)
def test_b1_engine_as_accurate_as_launch_path(cuda, name, layers, plen):
    """Teacher-forced decode steps: engine and launch-per-op path (both W8A8) against the unquantised
    bf16 model, each on its own KV cache filled by its own prefill."""
    from edgellm.engine.generate import Generator
    from edgellm.models.decoder import AttnCtx
    dev = torch.device("cuda", 0)
    cfg = _cfg(name, layers)
    ref = _model(cfg, dev, quant=False)
    model = _model(cfg, dev)
    g = torch.Generator().manual_seed(1)
    prompt = torch.randint(0, cfg.vocab_size, (1, plen), generator=g).to(dev)
    kvs = []
    for m in (ref, model, model):
        gen = Generator(m, max_batch=1, max_seq=512, use_graphs=False)
        gen.prefill(prompt)
        kvs.append(gen.kv)
    rope = model.rope_table(dev)
    err_e, err_l = [], []
    for s in range(4):
        pos = plen + s
        tok = torch.randint(0, cfg.vocab_size, (1, 1), generator=g).to(dev)
        sp = torch.full((1,), pos, dtype=torch.int32, device=dev)
        out = [m(tok, AttnCtx("decode", 1, 1, sp, sp + 1, pos + 1, kv.rows(0, 1), rope, b1=b1)).float()
               for m, kv, b1 in ((ref, kvs[0], False), (model, kvs[1], False), (model, kvs[2], True))]
        err_l.append(_rel(out[1], out[0]))
        err_e.append(_rel(out[2], out[0]))
    from edgellm.engine import b1_engine
    b1_engine.engine_for(model, kvs[2]).check()
    assert sum(err_e) <= 1.3 * sum(err_l) + 0.02, (err_e, err_l)


def test_b1_engine_generator_graphs(cuda):
    """Generator decode through the engine: the eager warm step, then graph capture + replay; the
    first sampled token (from the shared prefill) is identical, the rest are valid ids."""
    from edgellm.engine import SamplingParams
    from edgellm.engine.generate import Generator
    dev = torch.device("cuda", 0)
    cfg = _cfg("llama-2-7b", 2)
    model = _model(cfg, dev)
    sp = SamplingParams(max_new_tokens=24, do_sample=False, repetition_penalty=1.0)
    prompt = [[5, 17, 300, 42, 7, 1000, 12, 9]]
    res = {}
    for b1 in (False, True):
        gen = Generator(model, max_batch=1, max_seq=256)
        gen.b1 = b1
        r = gen.generate(prompt, sp, seed=0)
        res[b1] = r.tokens[0]
        if b1:
            assert len(gen._graphs) >= 1 and len(model._b1_engines) >= 1
    assert len(res[True]) == 24 and all(0 <= t < cfg.vocab_size for t in res[True])
    assert res[True][0] == res[False][0]


@pytest.mark.parametrize("name", ["llama-2-7b", "llama-3.2-1b"])
def test_b1_engine_deterministic_over_launches(cuda, name):
    """The same step launched 40 times (same token, same position: the append rewrites the same row
    with the same values) gives bit-identical outputs: no launch-to-launch race between the streams,
    the seams and the granule tags (a fresh tag every launch)."""
    from edgellm.engine import b1_engine
    dev = torch.device("cuda", 0)
    cfg, model, kv, g = _setup(name, 3, 150, dev)
    eng = b1_engine.engine_for(model, kv)
    x0 = model.embed[torch.tensor([7], device=dev)].contiguous()
    sp = torch.full((1,), 150, dtype=torch.int32, device=dev)
    ref = eng.run(x0, sp).clone()
    outs = [eng.run(x0, sp).clone() for _ in range(40)]
    torch.cuda.synchronize()
    eng.check()
    bad = [i for i, o in enumerate(outs) if not torch.equal(o, ref)]
    assert not bad, bad
