"""Batch-1 W8A8 decode of a whole Llama-family stack in one persistent launch (ops/csrc/b1_engine.hip).

The reference's own workload is single-stream generation (HF ``generate`` at batch 1,
Code/Base Models/combine_model_fp_updated.py:86-110), where every projection is a weight stream.
The launch-per-op decode path (models/decoder.py) runs five kernels per layer and loses ~20 us per
Llama-2-7B layer to their boundaries, ramps and tails.  This module lays the int8 weights out as one
contiguous stream per wave (workgroup = one CU, 4 waves) in the exact order the kernel consumes them,
so the weight stream runs across every projection and layer of a step while the dependency waits
overlap it.

Layout (``stream_layout``): every projection's output columns are cut into 16-column units (the
gate_up projection: 8 features = their 8 gate + 8 up rows), units spread evenly over the G CUs
(``unit_split``); each of a CU's 4 waves owns a quarter of K.  A fragment is 16 columns x 64 k, lane
l holding W[col 4 (l >> 2)..][k 16 (l & 3) .. +16], and wave w's stream is, for every layer, the
qkv / o / gate_up / down fragments of its CU's units, unit-major, its k-blocks in order.  The weight
bytes are a second copy of the model's int8 weights (6.5 GB at Llama-2-7B, of 288 GB): the prefill
and batched paths keep using the MFMA-packed originals.

Use: ``Generator`` turns it on for batch-1 decode when ``EDGELLM_B1_ENGINE`` is "1" and the model is
eligible (``eligible``); ``DecoderLM.forward`` then runs embedding -> ``B1Engine.run`` -> final norm +
LM head.  Concurrent use of two engines on one GPU is not allowed (each launch needs every CU):
``co_generate`` / ``LaneGenerator`` never enable it.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional, Tuple

import torch

from .. import ops

RING_DEPTHS = (24, 16)          # fragments in flight per wave (the kernel's D), largest that fits LDS
MAXK = 8                        # granules a thread sweeps in a norm seam (kernel B1_MAXK)
MAXCU = 8                       # units per CU and projection (kernel B1_MAXCU)
MAXA = 4                        # attention-output granules a thread sweeps (kernel B1_MAXA)
MAXH = 24                       # SwiGLU-output granules a thread sweeps (kernel B1_MAXH)


def enabled() -> bool:
    return os.environ.get("EDGELLM_B1_ENGINE", "0") == "1"


def unit_split(nu: int, G: int) -> torch.Tensor:
    """First unit of every CU (length G + 1): CU c owns units [u0[c], u0[c + 1]) (kernel u0_of)."""
    return torch.tensor([(c * nu) // G for c in range(G + 1)], dtype=torch.long)


def _why_not(model, G: int) -> Optional[str]:
    from ..quant.linear import W8A8Linear
    cfg = model.cfg
    if not (model.has_embed and model.has_head and model.first == 0 and model.last == cfg.num_layers):
        return "not a whole model"
    if cfg.norm != "rms" or cfg.act != "silu_glu" or cfg.parallel_residual or cfg.pos_emb != "rope":
        return "not a Llama-family block"
    HD = cfg.head_dim
    if HD not in (64, 128) or (cfg.rotary_dim or HD) != HD:
        return f"head_dim {HD} / partial rotary"
    if cfg.qkv_bias or cfg.o_bias or cfg.mlp_bias:
        return "projection biases"
    H, F, Hq, Hkv = cfg.hidden_size, cfg.intermediate_size, cfg.num_heads, cfg.num_kv_heads
    NQ = (Hq + 2 * Hkv) * HD
    if H % 256 or (Hq * HD) % 256 or F % 256 or Hq % Hkv or Hq > G or G > 512:
        return "shape"
    if -(-NQ // 16 // G) > MAXCU or -(-F // 8 // G) > MAXCU or -(-H // 16 // G) > MAXCU:
        return "too many units per CU"
    if G * -(-16 * -(-H // 16 // G) // 3) > 256 * MAXK or Hq * (HD // 64) * 12 > 256 * MAXA or \
            G * -(-8 * -(-F // 8 // G) // 3) > 256 * MAXH:
        return "too large for one seam sweep"
    for layer in model.layers:
        for lin in (layer.attn.qkv, layer.attn.o, layer.mlp.up, layer.mlp.down):
            if type(lin) is not W8A8Linear or lin.bias is not None:
                return "projections are not W8A8"
    if model.dtype != torch.bfloat16:
        return "not a bf16 model"
    return None


def eligible(model, G: Optional[int] = None) -> bool:
    if G is None:
        if not torch.cuda.is_available():
            return False
        G = torch.cuda.get_device_properties(model.device).multi_processor_count
    return _why_not(model, G) is None


def _phase_units(q: torch.Tensor, glu: bool) -> torch.Tensor:
    """Canonical int8 [N, K] -> [NU, 16, K] (gate_up [gate(F) | up(F)]: unit u = gate rows 8u..8u+7,
    then up rows 8u..8u+7)."""
    N, K = q.shape
    if glu:
        F = N // 2
        return torch.cat([q[:F].view(F // 8, 8, K), q[F:].view(F // 8, 8, K)], 1)
    return q.view(N // 16, 16, K)


def _fragments(wu: torch.Tensor) -> torch.Tensor:
    """[NU, 16, K] -> [NU, 4 waves, kbw, 1024] (lane l = 4 col + ksub holds W[col][64 kb + 16 ksub ..])."""
    NU, _, K = wu.shape
    kbw = K // 256
    f = wu.view(NU, 16, 4, kbw, 4, 16).permute(0, 2, 3, 1, 4, 5)
    return f.reshape(NU, 4, kbw, 1024)


def stream_layout(weights, H: int, F: int, NQ: int, QH: int, G: int, device=None) -> Tuple[torch.Tensor, int]:
    """Per-wave fragment streams [G, 4, fmax, 1024] int8 from the canonical int8 weights
    ``weights`` = [(qkv [NQ, H], o [H, QH], gate_up [2F, H], down [H, F])] per layer."""
    L = len(weights)
    NUq, NUh, NUf = NQ // 16, H // 16, F // 8
    uq, uh, uf = unit_split(NUq, G), unit_split(NUh, G), unit_split(NUf, G)
    nq, nh, nf = uq[1:] - uq[:-1], uh[1:] - uh[:-1], uf[1:] - uf[:-1]
    kbq, kbo, kbd = H // 256, QH // 256, F // 256
    # fragments of each phase per CU, and the phase offsets within a layer
    npq, npo, npg, npd = nq * kbq, nh * kbo, nf * kbq, nh * kbd
    per_layer = npq + npo + npg + npd
    fmax = int(per_layer.max()) * L
    ws = torch.empty(G * 4 * fmax, 1024, dtype=torch.int8, device=device)
    offs = (torch.zeros(G, dtype=torch.long), npq, npq + npo, npq + npo + npg)
    splits = (uq, uh, uf, uh)
    kbws = (kbq, kbo, kbq, kbd)
    owner = []
    for sp in splits:                                   # CU of every unit
        nu = int(sp[-1])
        owner.append(torch.repeat_interleave(torch.arange(G), sp[1:] - sp[:-1], output_size=nu))
    for l, mats in enumerate(weights):
        for ph, q in enumerate(mats):
            fr = _fragments(_phase_units(q.to(device), glu=ph == 2))            # [NU, 4, kbw, 1024]
            NU, kbw = fr.shape[0], kbws[ph]
            own = owner[ph]
            # stream position of (unit, wave, kb): CU base + layer l + phase offset + unit-major order
            base = own * 4 * fmax + l * per_layer[own] + offs[ph][own] + (torch.arange(NU) - splits[ph][own]) * kbw
            idx = (base[:, None, None] + torch.arange(4)[None, :, None] * fmax + torch.arange(kbw)[None, None, :])
            ws[idx.reshape(-1).to(ws.device)] = fr.reshape(-1, 1024)
    return ws.view(G, 4, fmax, 1024), fmax


class B1Weights:
    """The per-model part: weight streams, scales, norm weights, RoPE table, dimensions."""

    @torch.no_grad()
    def __init__(self, model, G: int):
        cfg = model.cfg
        why = _why_not(model, G)
        assert why is None, f"batch-1 engine: {why}"
        dev = model.device
        self.G = G
        self.L, self.H, self.F = cfg.num_layers, cfg.hidden_size, cfg.intermediate_size
        self.Hq, self.Hkv, self.HD = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
        self.NQ = (self.Hq + 2 * self.Hkv) * self.HD
        self.eps, self.scale = float(cfg.norm_eps), 1.0 / math.sqrt(self.HD)
        mats, sq, so, sg, sd, g1, g2 = [], [], [], [], [], [], []
        for layer in model.layers:
            qkv, o, up, down = layer.attn.qkv, layer.attn.o, layer.mlp.up, layer.mlp.down
            cq, cs, _ = qkv.canonical()
            co, cso, _ = o.canonical()
            cu, csu, _ = up.canonical()
            cd, csd, _ = down.canonical()
            mats.append((cq, co, cu, cd))
            sq.append(cs.float()); so.append(cso.float()); sg.append(csu.float()); sd.append(csd.float())
            g1.append(layer.norm1.weight.detach()); g2.append(layer.norm2.weight.detach())
        self.ws, self.fmax = stream_layout(mats, self.H, self.F, self.NQ, self.Hq * self.HD, G, dev)
        self.sw_q, self.sw_o = torch.stack(sq).contiguous(), torch.stack(so).contiguous()
        self.sw_gu, self.sw_d = torch.stack(sg).contiguous(), torch.stack(sd).contiguous()
        self.gam1 = torch.stack(g1).to(torch.bfloat16).contiguous()
        self.gam2 = torch.stack(g2).to(torch.bfloat16).contiguous()
        self.rope = model.rope_table(dev).contiguous()
        self.version = _weights_version(model)

    def nbytes(self) -> int:
        return self.ws.numel()


def _weights_version(model) -> tuple:
    return tuple(int(b._version) for layer in model.layers
                 for b in (layer.attn.qkv.w_packed, layer.attn.o.w_packed, layer.mlp.up.w_packed,
                           layer.mlp.down.w_packed, layer.norm1.weight, layer.norm2.weight))


class B1Engine:
    """One model + one KV cache (batch row 0): granule buffers, control words and the output."""

    @torch.no_grad()
    def __init__(self, w: B1Weights, kv, device):
        assert not getattr(kv, "quantized", False) and kv.k.dtype == torch.bfloat16, "bf16 KV cache"
        assert kv.first == 0 and kv.last == w.L and kv.k.is_contiguous() and kv.v.is_contiguous()
        self.w, self.kv = w, kv
        G, L, H, F, Hq, HD = w.G, w.L, w.H, w.F, w.Hq, w.HD
        nmax = lambda nu: -(-nu // G)                                  # noqa: E731
        self.gpc_x = -(-16 * nmax(H // 16) // 3)
        self.gpc_q = -(-16 * nmax(w.NQ // 16) // 3)
        self.gpc_h = -(-8 * nmax(F // 8) // 3)
        z = lambda *s: torch.zeros(*s, dtype=torch.int64, device=device)   # noqa: E731
        self.gx, self.gr = z(L, G, self.gpc_x), z(L, G, self.gpc_x)
        self.gq, self.gh = z(L, G, self.gpc_q), z(L, G, self.gpc_h)
        self.ga = z(L, Hq, HD // 64, 12)
        self.ctl = torch.zeros(4, dtype=torch.int32, device=device)
        self.xout = torch.zeros(1, H, dtype=torch.bfloat16, device=device)
        S = kv.k.shape[3]
        r16 = lambda n: (n + 15) // 16 * 16                              # noqa: E731
        self.xqb = r16(max(H, Hq * HD, F))
        self.sxn = r16(max(H, Hq * HD, F) // 64 + 4)
        self.scb = r16(max(2 * F, 4 * H, (9 * HD + S + 64) * 4 + 160))
        C = ops.ext()
        self.D = None
        for D in RING_DEPTHS:
            lds = C.b1_lds_bytes(D, self.xqb, self.sxn, self.scb)
            if lds <= 160 * 1024:
                self.D, self.lds = D, lds
                break
        assert self.D is not None, "batch-1 engine: LDS"
        B, Hkv = kv.k.shape[1], kv.k.shape[2]
        self.kv_l, self.kv_h = B * Hkv * S * HD, S * HD

    def run(self, x0: torch.Tensor, pos: torch.Tensor, stamps: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x0: bf16 [1, H] embedding of the token; pos: int32 device tensor whose [0] is its position.
        Returns the residual stream after the last layer, bf16 [1, H] (an engine-owned buffer).
        ``stamps``: int64 [G, L, 24] receives each CU's phase-boundary clock (tools/b1_profile.py)."""
        w = self.w
        ops.ext().b1_decode(
            [w.ws, w.sw_q, w.sw_o, w.sw_gu, w.sw_d, w.gam1, w.gam2, w.rope, x0.contiguous(), self.xout, self.kv.k,
             self.kv.v, pos, self.gx, self.gq, self.ga, self.gr, self.gh, self.ctl] +
            ([] if stamps is None else [stamps]),
            [w.fmax, self.kv_l, self.kv_h, w.L, w.H, w.Hq, w.Hkv, w.F, w.NQ, self.gpc_x, self.gpc_q, self.gpc_h,
             self.xqb, self.sxn, self.scb, w.G, self.D, w.HD, self.lds],
            w.eps, w.scale)
        return self.xout

    def check(self) -> None:
        """Raise if a launch gave up on a seam (bounded spins; ctl[2] names the seam)."""
        ctl = self.ctl.tolist()
        if ctl[1] or ctl[2]:
            # a launch that gave up leaves counters / salt out of step: start the protocol state over
            for b in (self.ctl, self.gx, self.gq, self.ga, self.gr, self.gh):
                b.zero_()
            raise RuntimeError(f"batch-1 engine: a launch gave up waiting (seam code {ctl[2]})")


def engine_for(model, kv) -> Optional[B1Engine]:
    """The model's engine for this KV cache (built on first use; rebuilt if the weights changed)."""
    if not (ops.available() and kv.k.is_cuda and kv.k.shape[1] >= 1):
        return None
    G = torch.cuda.get_device_properties(kv.k.device).multi_processor_count
    if _why_not(model, G) is not None or getattr(kv, "quantized", False) or kv.first != 0:
        return None
    w = getattr(model, "_b1_weights", None)
    if w is None or w.G != G or w.version != _weights_version(model):
        w = model._b1_weights = B1Weights(model, G)
        model._b1_engines = {}
    engines: Dict[int, B1Engine] = model.__dict__.setdefault("_b1_engines", {})
    key = kv.k.data_ptr()
    e = engines.get(key)
    if e is None or e.kv is not kv:
        e = engines[key] = B1Engine(w, kv, kv.k.device)
    return e
