import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, edgellm
from edgellm import ops
for D in (64, 128, 256):
    B, Hkv, S, T = 3, 2, 40, 7
    g = torch.Generator().manual_seed(D)
    src = torch.randn(B, Hkv, S, D, generator=g).to(torch.bfloat16)
    start = torch.tensor([0, 5, 30], dtype=torch.int32)
    c_r = torch.zeros(B, Hkv, S, D, dtype=torch.int8); s_r = torch.zeros(B, Hkv, S)
    ops.kv_quant_append(src, start, T, c_r, s_r)
    c_g = torch.zeros_like(c_r).cuda(); s_g = torch.zeros_like(s_r).cuda()
    ops.kv_quant_append(src.cuda(), start.cuda(), T, c_g, s_g)
    torch.cuda.synchronize()
    d = (c_g.cpu().int() - c_r.int())
    nz = d.nonzero()
    print(D, "mismatches", nz.shape[0], "maxabs", d.abs().max().item(), "scale maxrel", ((s_g.cpu()-s_r).abs()/(s_r.abs()+1e-12)).max().item())
    print(nz[:10].tolist())
    if nz.shape[0]:
        b,h,p,e = nz[0].tolist()
        print("gpu", c_g[b,h,p,:8].tolist(), "ref", c_r[b,h,p,:8].tolist(), "src", src[b,h,p,:8].tolist())
