"""BERT-style bidirectional encoder (all-MiniLM-L6-v2 class) for the evaluation harness.

The reference embeds texts with ``SentenceTransformer('all-MiniLM-L6-v2')`` and compares them
with ``util.pytorch_cos_sim`` (combine_model_fp_updated.py:70-73,179) — mean pooling over
token embeddings, L2-normalised.  BERTScore (K15) uses the same kind of encoder's contextual
token embeddings.  This encoder reads HF ``BertModel`` checkpoints (safetensors) or is
random-initialised; it is off the generation hot path ("optional"), so attention
uses torch SDPA while the LayerNorms go through edgellm.ops.
"""
from __future__ import annotations

import glob
import json
import os
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .configs import ModelConfig, PRESETS


class BertLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype, device):
        super().__init__()
        h, f = cfg.hidden_size, cfg.intermediate_size
        mk = lambda i, o: nn.Linear(i, o, dtype=dtype, device=device)  # noqa: E731
        self.q, self.k, self.v, self.o = mk(h, h), mk(h, h), mk(h, h), mk(h, h)
        self.ln1 = nn.LayerNorm(h, eps=cfg.norm_eps, dtype=dtype, device=device)
        self.up, self.down = mk(h, f), mk(f, h)
        self.ln2 = nn.LayerNorm(h, eps=cfg.norm_eps, dtype=dtype, device=device)
        self.heads = cfg.num_heads

    def forward(self, x, mask):
        B, T, H = x.shape
        d = H // self.heads
        q, k, v = (t(x).view(B, T, self.heads, d).transpose(1, 2) for t in (self.q, self.k, self.v))
        a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
        a = self.o(a.transpose(1, 2).reshape(B, T, H))
        x = _ln(self.ln1, a, x)                     # post-LN: LN(x + attn)
        m = self.down(F.gelu(self.up(x)))
        return _ln(self.ln2, m, x)


def _ln(ln: nn.LayerNorm, x, residual):
    if x.is_cuda and x.dtype == torch.bfloat16:
        y, _ = ops.layer_norm(x.reshape(-1, x.shape[-1]).contiguous(), ln.weight, ln.bias, ln.eps,
                              residual.reshape(-1, x.shape[-1]).contiguous())
        return y.view_as(x)
    return ln(x + residual)


class BertEncoder(nn.Module):
    def __init__(self, cfg: ModelConfig = PRESETS["minilm-l6"], dtype=torch.float32, device=None,
                 type_vocab: int = 2):
        super().__init__()
        self.cfg = cfg
        h = cfg.hidden_size
        self.word = nn.Embedding(cfg.vocab_size, h, dtype=dtype, device=device)
        self.pos = nn.Embedding(cfg.max_position_embeddings, h, dtype=dtype, device=device)
        self.typ = nn.Embedding(type_vocab, h, dtype=dtype, device=device)
        self.ln = nn.LayerNorm(h, eps=cfg.norm_eps, dtype=dtype, device=device)
        self.layers = nn.ModuleList([BertLayer(cfg, dtype, device) for _ in range(cfg.num_layers)])

    def forward(self, ids: torch.Tensor, attn: Optional[torch.Tensor] = None) -> torch.Tensor:
        """ids [B, T] -> token embeddings [B, T, H]"""
        B, T = ids.shape
        if attn is None:
            attn = torch.ones_like(ids)
        pos = torch.arange(T, device=ids.device)[None]
        x = self.ln(self.word(ids) + self.pos(pos) + self.typ(torch.zeros_like(ids)))
        mask = attn[:, None, None, :].bool()
        for layer in self.layers:
            x = layer(x, mask)
        return x

    @torch.no_grad()
    def sentence_embedding(self, ids: torch.Tensor, attn: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Mean pooling over valid tokens, L2-normalised (sentence-transformers MiniLM recipe)."""
        if attn is None:
            attn = torch.ones_like(ids)
        tok = self.forward(ids, attn).float()
        m = attn[..., None].float()
        emb = (tok * m).sum(1) / m.sum(1).clamp_min(1e-9)
        return F.normalize(emb, dim=-1)


_HF_MAP = {"embeddings.word_embeddings.weight": "word.weight", "embeddings.position_embeddings.weight": "pos.weight",
           "embeddings.token_type_embeddings.weight": "typ.weight", "embeddings.LayerNorm.weight": "ln.weight",
           "embeddings.LayerNorm.bias": "ln.bias"}
_HF_LAYER = {"attention.self.query": "q", "attention.self.key": "k", "attention.self.value": "v",
             "attention.output.dense": "o", "attention.output.LayerNorm": "ln1", "intermediate.dense": "up",
             "output.dense": "down", "output.LayerNorm": "ln2"}


def load_bert(path: str, dtype=torch.float32, device=None) -> BertEncoder:
    from safetensors import safe_open
    from .configs import from_hf_config
    with open(os.path.join(path, "config.json")) as f:
        cfg = from_hf_config(json.load(f))
    enc = BertEncoder(cfg, dtype, device)
    sd = {}
    for fn in sorted(glob.glob(os.path.join(path, "*.safetensors"))):
        with safe_open(fn, framework="pt") as sf:
            for k in sf.keys():
                kk = k[5:] if k.startswith("bert.") else k
                if kk in _HF_MAP:
                    sd[_HF_MAP[kk]] = sf.get_tensor(k)
                elif kk.startswith("encoder.layer."):
                    _, _, i, rest = kk.split(".", 3)
                    for hf, ours in _HF_LAYER.items():
                        if rest.startswith(hf + "."):
                            sd[f"layers.{i}.{ours}.{rest[len(hf) + 1:]}"] = sf.get_tensor(k)
    missing, _ = enc.load_state_dict(sd, strict=False)
    if missing:
        raise KeyError(f"BERT checkpoint missing {missing[:5]}")
    return enc.eval()
