#!/usr/bin/env python
"""Where a batch-1 engine step spends its time: per-CU phase-boundary clocks (s_memrealtime, 100 MHz)
recorded by the kernel (ops/csrc/b1_engine.hip, B1Params.stamps), averaged over layers and steps.

    python tools/b1_profile.py [--model llama-2-7b] [--layers 32] [--steps 20] [--out stamps.json]
"""
import argparse
import dataclasses
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

PH = ["qkv seam", "qkv stream", "qkv epilogue", "attention", "o seam", "o stream", "o epilogue", "gu seam",
      "gu stream", "gu epilogue", "down seam", "down stream", "down epilogue"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-2-7b")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--plen", type=int, default=128)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import edgellm  # noqa: F401
    from edgellm.engine import b1_engine
    from edgellm.engine.generate import Generator
    from edgellm.models import build_model, get_config
    from edgellm.quant import quantize_model
    dev = torch.device("cuda", 0)
    cfg = dataclasses.replace(get_config(args.model), num_layers=args.layers)
    model = quantize_model(build_model(cfg, device=dev, seed=0), "w8a8_smoothquant")
    gen = Generator(model, max_batch=1, max_seq=args.plen + args.steps + 8, use_graphs=False)
    g = torch.Generator().manual_seed(1)
    gen.prefill(torch.randint(0, cfg.vocab_size, (1, args.plen), generator=g).to(dev))
    eng = b1_engine.engine_for(model, gen.kv)
    G, L = eng.w.G, eng.w.L
    st = torch.zeros(G, L, 24, dtype=torch.int64, device=dev)
    x0 = model.embed[:1].contiguous()
    acc, walls = [], []
    for s in range(args.steps + 3):
        pos = torch.full((1,), args.plen + s, dtype=torch.int32, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.run(x0, pos, st)
        e1.record()
        torch.cuda.synchronize()
        eng.check()
        if s >= 3:
            acc.append(st.clone().cpu())
            walls.append(e0.elapsed_time(e1))
    a = torch.stack(acc).double() * 10e-3                      # us
    d = a[..., 1:14] - a[..., 0:13]                              # [steps, G, L, 13] phase durations
    res = {"wall_ms_mean": sum(walls) / len(walls), "model": args.model, "layers": L, "G": G,
           "layer_us_cu0": float((a[:, 0, 1:, 0] - a[:, 0, :-1, 0]).mean()),
           "phases_us": {}}
    Hq = cfg.num_heads
    for i, nm in enumerate(PH):
        res["phases_us"][nm] = {"attention CUs mean": round(float(d[:, :Hq, :, i].mean()), 2),
                                "other CUs mean": round(float(d[:, Hq:, :, i].mean()), 2),
                                "max over CUs (mean over layers)": round(float(d[:, :, :, i].amax(1).mean()), 2)}
    res["layer_span_us"] = round(float((a[:, :, -1, 13] - a[:, :, 0, 0]).mean() / L), 2)
    # attention sub-phases (attention CUs): qkv sweep, RoPE + scores, softmax, P.V, quantise + publish
    at = a[:, :Hq]
    sub = [("q/k/v sweep", 3, 14), ("rope + scores", 14, 15), ("softmax", 15, 16), ("P.V", 16, 17), ("quantise + publish", 17, 4)]
    res["attention_us"] = {nm: round(float((at[..., j] - at[..., i]).mean()), 2) for nm, i, j in sub}
    dsub = [("sweep", 10, 18), ("h to LDS + barrier", 18, 19), ("group quant", 19, 20), ("scale pin + barrier", 20, 11)]
    res["down_seam_us"] = {nm: round(float((a[..., j] - a[..., i]).mean()), 2) for nm, i, j in dsub}
    # each seam's cost after its LAST producer published: consumer seam end - max over producers
    seams = {"qkv seam (x)": (13, 1, -1), "o seam (attention)": (4, 5, 0), "gu seam (h2)": (7, 8, 0),
             "down seam (h)": (10, 11, 0)}
    res["seam_after_last_publish_us"] = {}
    for nm, (pi, ci, dl) in seams.items():
        if dl == -1:
            prod = a[:, :, :-1, pi].amax(1)            # [steps, L-1]: layer l's x published in layer l - 1
            cons = a[:, :, 1:, ci]                     # [steps, G, L-1]
        else:
            prod = (a[:, :Hq, :, pi] if pi == 4 else a[:, :, :, pi]).amax(1)
            cons = a[:, :, :, ci]
        res["seam_after_last_publish_us"][nm] = {
            "mean": round(float((cons - prod[:, None]).mean()), 2),
            "max": round(float((cons - prod[:, None]).amax(1).mean()), 2)}
        res["seam_producer_skew_us"] = res.get("seam_producer_skew_us", {})
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
