#!/usr/bin/env python
"""Stage-by-stage check of the batch-1 persistent decode engine (ops/csrc/b1_engine.hip).

Runs one decode step of a SmoothQuant W8A8 Llama-shaped model through the engine, then re-computes
every stage in fp32 torch from the canonical int8 weights with the engine's documented numerics and
compares it with what the engine published (its granule buffers hold the last launch's values):
qkv, the int8 attention output + scales, h2 = x + o, the SwiGLU output, the layer output.  Also
prints the launch-per-op path's final hidden for the same step.

    python tools/b1_debug.py [--model llama-2-7b] [--layers 1] [--plen 40]
"""
import argparse
import dataclasses
import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def unpack3(buf, G, gpc, counts, n):
    """granule blocks [G, gpc] of 3 bf16 each -> values [n] (block c holds counts[c] values)."""
    out = torch.zeros(n, dtype=torch.float32)
    b = buf.cpu().view(torch.int64)
    v0 = 0
    for c in range(G):
        for j in range((counts[c] + 2) // 3):
            g = int(b[c, j]) & ((1 << 64) - 1)
            for e in range(3):
                if 3 * j + e < counts[c]:
                    u = (g >> (16 * e)) & 0xFFFF
                    out[v0 + 3 * j + e] = struct.unpack('<f', struct.pack('<I', u << 16))[0]
        v0 += counts[c]
    return out


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def bf(x):
    return x.to(torch.bfloat16).float()


def quant_tok(y):
    am = y.abs().max().clamp_min(1e-8)
    s = am / 127
    return torch.round(y / s).clamp(-127, 127), s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-2-7b")
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--plen", type=int, default=40)
    ap.add_argument("--ref", action="store_true", help="the comparison path runs the torch reference ops on the GPU")
    args = ap.parse_args()
    import edgellm  # noqa: F401
    from edgellm.engine import b1_engine
    from edgellm.engine.generate import Generator
    from edgellm.models import build_model, get_config
    from edgellm.models.decoder import AttnCtx
    from edgellm.quant import quantize_model
    dev = torch.device("cuda", 0)
    cfg = dataclasses.replace(get_config(args.model), num_layers=args.layers, vocab_size=4096,
                              max_position_embeddings=1024)
    model = quantize_model(build_model(cfg, device=dev, seed=3), "w8a8_smoothquant")
    gen = Generator(model, max_batch=1, max_seq=512, use_graphs=False)
    g = torch.Generator().manual_seed(1)
    plen = args.plen
    gen.prefill(torch.randint(0, cfg.vocab_size, (1, plen), generator=g).to(dev))
    kv = gen.kv
    k_before, v_before = kv.k.clone(), kv.v.clone()
    tok = torch.randint(0, cfg.vocab_size, (1, 1), generator=g).to(dev)
    sp = torch.full((1,), plen, dtype=torch.int32, device=dev)
    rope = model.rope_table(dev)
    # launch-per-op path first (on a copy of the cache), then the engine
    kv_ref = type(kv)(cfg, 1, 512, device=dev)
    kv_ref.k.copy_(kv.k)
    kv_ref.v.copy_(kv.v)
    cap = {}
    hooks = []
    from edgellm.models.layers import PartialSum, QAct

    def _val(x):
        if isinstance(x, QAct):
            q, sc = x.q.float().reshape(-1), x.scale.float()
            if sc.dim() == 2:                        # per-(token, 64): [G64, Mpad]
                return (q.view(-1, 64) * sc[:, :1]).reshape(-1)
            return q * sc.reshape(-1)[0]
        if isinstance(x, PartialSum):
            return x.parts.float().sum(0).reshape(-1)
        if isinstance(x, tuple):
            return _val(x[0])
        return x.float().reshape(-1)
    for l, layer in enumerate(model.layers):
        for nm, mod in (("qkv", layer.attn.qkv), ("o", layer.attn.o), ("down", layer.mlp.down)):
            hooks.append(mod.register_forward_hook(
                lambda m, i, o, k=f"L{l}.{nm}": cap.update({k + ".in": _val(i[0]), k + ".out": _val(o)})))
    from edgellm import ops as _ops
    _ops._REF_ON_GPU = args.ref
    ref_hidden = model(tok, AttnCtx("decode", 1, 1, sp, sp + 1, plen + 1, kv_ref.rows(0, 1), rope), logits="hidden")
    _ops._REF_ON_GPU = False
    for h in hooks:
        h.remove()
    eng = b1_engine.engine_for(model, kv)
    x0 = model.embed[tok.reshape(-1)].contiguous()
    xout = eng.run(x0, sp).clone()
    torch.cuda.synchronize()
    eng.check()
    w = eng.w
    G, H, F, Hq, Hkv, HD, NQ = w.G, w.H, w.F, w.Hq, w.Hkv, w.HD, w.NQ
    split = b1_engine.unit_split
    cnt_h = [16 * int(n) for n in split(H // 16, G).diff()]
    cnt_q = [16 * int(n) for n in split(NQ // 16, G).diff()]
    cnt_f = [8 * int(n) for n in split(F // 8, G).diff()]
    res = {}
    x = x0.float().reshape(-1)
    for l, layer in enumerate(model.layers):
        qkv_w, o_w, up_w, dn_w = (m.canonical() for m in (layer.attn.qkv, layer.attn.o, layer.mlp.up, layer.mlp.down))
        # qkv
        r = torch.rsqrt(x.pow(2).mean() + w.eps)
        y = x * layer.norm1.weight.float()
        q8, s = quant_tok(y * r)
        qkv = bf((q8 @ qkv_w[0].float().t()) * s * qkv_w[1].float())
        e_qkv = unpack3(eng.gq[l], G, eng.gpc_q, cnt_q, NQ)
        res[f"L{l}.qkv"] = rel(e_qkv, qkv.cpu())
        if f"L{l}.qkv.out" in cap:
            res[f"L{l}.qkv_launch_vs_emu"] = rel(cap[f"L{l}.qkv.out"].cpu(), qkv.cpu())
        qkv = e_qkv.to(dev)                                         # continue from the engine's values
        # attention (head-major cache [Hkv, S, HD] of row 0)
        pos = plen
        q = qkv[:Hq * HD].view(Hq, HD)
        k = qkv[Hq * HD:(Hq + Hkv) * HD].view(Hkv, HD)
        v = qkv[(Hq + Hkv) * HD:].view(Hkv, HD)
        cs = rope[pos]
        c_, s_ = cs[:, 0], cs[:, 1]
        rot = lambda t: torch.cat([t[:, :HD // 2] * c_ - t[:, HD // 2:] * s_, t[:, HD // 2:] * c_ + t[:, :HD // 2] * s_], 1)  # noqa
        qr, kr = bf(rot(q)), bf(rot(k))
        kc = k_before[l, 0].float().clone()
        vc = v_before[l, 0].float().clone()
        kc[:, pos], vc[:, pos] = kr, v
        res[f"L{l}.k_append"] = rel(kv.k[l, 0, :, pos].float(), kr)
        res[f"L{l}.v_append"] = rel(kv.v[l, 0, :, pos].float(), v)
        grp = Hq // Hkv
        att = []
        for h in range(Hq):
            sc = (kc[h // grp, :pos + 1] @ qr[h]) * w.scale
            p = torch.softmax(sc, 0)
            att.append(p @ vc[h // grp, :pos + 1])
        att = bf(torch.cat(att))
        a8 = att.view(-1, 64)
        sa = a8.abs().amax(1).clamp_min(1e-8) / 127
        aq = torch.round(a8 / sa[:, None]).clamp(-127, 127)
        gaw = eng.ga[l].reshape(-1, 12).cpu()
        e_aq, e_sa = torch.zeros_like(aq).cpu(), torch.zeros_like(sa).cpu()
        for gi in range(gaw.shape[0]):
            byts = []
            for j in range(11):
                gval = int(gaw[gi, j]) & ((1 << 48) - 1)
                byts += [(gval >> (8 * b)) & 0xFF for b in range(6 if j < 10 else 4)]
            e_aq[gi] = torch.tensor([b - 256 if b > 127 else b for b in byts], dtype=torch.float32)
            e_sa[gi] = struct.unpack('<f', struct.pack('<I', int(gaw[gi, 11]) & 0xFFFFFFFF))[0]
        res[f"L{l}.att_q"] = rel(e_aq * e_sa[:, None], (aq * sa[:, None]).cpu())
        if f"L{l}.o.in" in cap:
            res[f"L{l}.att_launch_vs_emu"] = rel(cap[f"L{l}.o.in"].cpu(), (aq * sa[:, None]).reshape(-1).cpu())
            res[f"L{l}.att_launch_vs_engine"] = rel(cap[f"L{l}.o.in"].cpu(), (e_aq * e_sa[:, None]).reshape(-1))
        aq, sa = e_aq.to(dev), e_sa.to(dev)
        # o: grouped scales
        ow = o_w[0].float().view(H, -1, 64)                          # [N, G64, 64]
        o = (torch.einsum("ngk,gk->ng", ow, aq) * sa[None]).sum(1) * o_w[1].float()
        h2 = bf(o + x)
        e_h2 = unpack3(eng.gr[l], G, eng.gpc_x, cnt_h, H)
        res[f"L{l}.h2"] = rel(e_h2, h2.cpu())
        if f"L{l}.o.out" in cap:
            res[f"L{l}.o_launch_vs_emu(o only)"] = rel(cap[f"L{l}.o.out"].cpu(), o.cpu())
        h2 = e_h2.to(dev)
        # gate_up + SwiGLU
        r2 = torch.rsqrt(h2.pow(2).mean() + w.eps)
        q8, s = quant_tok(h2 * layer.norm2.weight.float() * r2)
        gu = (q8 @ up_w[0].float().t()) * s * up_w[1].float()
        gg, uu = bf(gu[:F]), bf(gu[F:])
        hh = bf(gg / (1 + torch.exp(-gg)) * uu)
        e_h = unpack3(eng.gh[l], G, eng.gpc_h, cnt_f, F)
        res[f"L{l}.h"] = rel(e_h, hh.cpu())
        if f"L{l}.down.in" in cap:
            h8e = hh.view(-1, 64)
            hse = h8e.abs().amax(1).clamp_min(1e-8) / 127
            hqe = (torch.round(h8e / hse[:, None]).clamp(-127, 127) * hse[:, None]).reshape(-1)
            res[f"L{l}.hq_launch_vs_emu"] = rel(cap[f"L{l}.down.in"].cpu(), hqe.cpu())
            hf = (gg / (1 + torch.exp(-gg)) * uu).view(-1, 64)             # fp32 h (the reference quantises it)
            hsf = hf.abs().amax(1).clamp_min(1e-8) / 127
            hqf = (torch.round(hf / hsf[:, None]).clamp(-127, 127) * hsf[:, None]).reshape(-1)
            res[f"L{l}.hq_launch_vs_emu_fp32h"] = rel(cap[f"L{l}.down.in"].cpu(), hqf.cpu())
            res[f"L{l}.hq_bf16h_vs_fp32h"] = rel(hqe.cpu(), hqf.cpu())
        hh = e_h.to(dev)
        # down: grouped scales per 64 features
        h8 = hh.view(-1, 64)
        hs = h8.abs().amax(1).clamp_min(1e-8) / 127
        hq = torch.round(h8 / hs[:, None]).clamp(-127, 127)
        dw = dn_w[0].float().view(H, -1, 64)
        dn = (torch.einsum("ngk,gk->ng", dw, hq) * hs[None]).sum(1) * dn_w[1].float()
        x = bf(dn + h2)
    res["xout"] = rel(xout.float().reshape(-1), x)
    fn = model.final_norm
    eng_hidden, _ = fn(xout, None)
    res["final_hidden_vs_launch_path"] = rel(eng_hidden.float(), ref_hidden.float())
    emu_hidden, _ = fn(x.to(torch.bfloat16).view(1, -1), None)
    res["emulation_vs_launch_path"] = rel(emu_hidden.float(), ref_hidden.float())
    print(json.dumps({k: round(v, 5) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
