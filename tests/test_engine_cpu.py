import torch

from edgellm.engine import Generator, KVCache, SamplingParams
from edgellm.models import AttnCtx, build_model, tiny


def _full_logits(model, ids):
    T = ids.shape[1]
    kv = KVCache(model.cfg, 1, T, dtype=model.dtype)
    sp = torch.zeros(1, dtype=torch.int32)
    return model(ids, AttnCtx("prefill", 1, T, sp, sp + T, T, kv, model.rope_table()), logits="last")


def test_greedy_generation_matches_recompute():
    cfg = tiny("llama")
    m = build_model(cfg, dtype=torch.float32, seed=5)
    gen = Generator(m, max_batch=2, max_seq=64)
    prompt = [3, 14, 15, 92, 65]
    res = gen.generate([prompt], SamplingParams(max_new_tokens=10, do_sample=False, repetition_penalty=1.0))
    ids = list(prompt)
    for _ in range(10):
        ids.append(int(_full_logits(m, torch.tensor([ids])).argmax(-1)))
    assert res.tokens[0] == ids[len(prompt):]


def test_sampling_is_seeded_and_batched():
    cfg = tiny("gpt_neox")
    m = build_model(cfg, dtype=torch.float32, seed=5)
    gen = Generator(m, max_batch=4, max_seq=64)
    sp = SamplingParams(max_new_tokens=12, temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1)
    a = gen.generate([[1, 2, 3], [4, 5, 6]], sp, seed=11)
    b = gen.generate([[1, 2, 3], [4, 5, 6]], sp, seed=11)
    c = gen.generate([[1, 2, 3], [4, 5, 6]], sp, seed=12)
    assert a.tokens == b.tokens and a.tokens != c.tokens
    # variable-length prompts in one batch == each alone (greedy)
    gp = SamplingParams(max_new_tokens=6, do_sample=False)
    both = gen.generate([[7, 8, 9, 10], [11, 12]], gp)
    one = gen.generate([[7, 8, 9, 10]], gp)
    two = gen.generate([[11, 12]], gp)
    assert both.tokens == [one.tokens[0], two.tokens[0]]


def test_eos_stop_and_tps_definitions():
    cfg = tiny("phi")
    m = build_model(cfg, dtype=torch.float32, seed=9)
    gen = Generator(m, max_batch=1, max_seq=64, eos_check_every=2)
    free = gen.generate([[5, 6, 7]], SamplingParams(max_new_tokens=12, do_sample=False))
    eos = free.tokens[0][3]
    res = gen.generate([[5, 6, 7]], SamplingParams(max_new_tokens=12, do_sample=False), eos_token_id=eos)
    assert res.tokens[0][-1] == eos and len(res.tokens[0]) == free.tokens[0].index(eos) + 1
    assert res.tps_incl_prompt() > res.tps_generated() > 0


def test_lane_generator_matches_independent_generators():
    """LaneGenerator deals prompts to lanes in contiguous chunks, seeds lane i with seed + 7919 i,
    and each lane decodes exactly as a standalone Generator would."""
    from edgellm.engine.generate import LaneGenerator
    cfg = tiny("llama")
    m = build_model(cfg, dtype=torch.float32, seed=5)
    prompts = [[3, 14, 15, 92, 65], [2, 7, 1, 8, 2], [1, 4, 1, 4, 2], [9, 9, 8, 7, 6]]
    sp = SamplingParams(max_new_tokens=8, temperature=0.7, top_k=20, top_p=0.9, repetition_penalty=1.1)
    lg = LaneGenerator(m, lanes=2, max_batch=2, max_seq=32)
    lg.start(prompts, sp, seed=11)
    lg.step(7)
    got = [r.tokens for r in lg.collect()]
    for i in range(2):
        ref = Generator(m, max_batch=2, max_seq=32).generate(prompts[2 * i:2 * i + 2], sp, seed=11 + 7919 * i)
        assert got[i] == ref.tokens


def test_ragged_batched_prefill_matches_one_at_a_time():
    """Unequal prompts prefill in ONE right-padded pass (AttnCtx.last_pos): greedy tokens and the
    sampled stream equal each prompt generated alone, for every decoder family."""
    prompts = [[3, 14, 15, 92, 65, 35, 89], [7, 1], [22, 4, 9, 9, 31], [5]]
    for arch in ("llama", "gpt_neox", "phi", "gpt2"):
        m = build_model(tiny(arch), dtype=torch.float32, seed=7)
        sp = SamplingParams(max_new_tokens=8, do_sample=False, repetition_penalty=1.1)
        batched = Generator(m, max_batch=4, max_seq=64)
        calls = []
        orig = batched.prefill
        batched.prefill = lambda *a, **k: calls.append(a[0].shape) or orig(*a, **k)
        res = batched.generate(prompts, sp)
        assert len(calls) == 1 and tuple(calls[0]) == (4, 7), calls     # one pass, padded to the longest
        for p, toks in zip(prompts, res.tokens):
            alone = Generator(m, max_batch=1, max_seq=64).generate([p], sp)
            assert toks == alone.tokens[0], arch


def test_sample_advance_is_sample_then_decode_advance():
    """ops.sample_advance (the decode step's sampler + bookkeeping) == ops.sample followed by
    ops.decode_advance on the CPU path; the GPU fused launch is pinned against the same pair in
    tests/test_kernels_gpu.py::test_sample_advance_matches_sample_then_advance."""
    from edgellm import ops
    g = torch.Generator().manual_seed(0)
    B, V = 3, 97
    mk = lambda: dict(tok=torch.zeros(B, dtype=torch.long), out=torch.zeros(B, 4, dtype=torch.long),  # noqa: E731
                      step=torch.tensor([0]), pos=torch.tensor([5, 6, 7], dtype=torch.int32),
                      lens=torch.tensor([6, 7, 8], dtype=torch.int32), rng=torch.tensor([11, 0], dtype=torch.int32),
                      seen=torch.zeros(B, V, dtype=torch.uint8))
    a, b = mk(), mk()
    ctr = torch.zeros(1, dtype=torch.int32)
    for _ in range(3):
        logits = torch.randn(B, V, generator=g)
        nxt = ops.sample(logits, a["seen"], 0.8, 10, 0.9, 1.1, a["rng"], True)
        ops.decode_advance(nxt, a["tok"], a["out"], a["step"], a["pos"], a["lens"], a["rng"])
        nb = ops.sample_advance(logits, b["seen"], 0.8, 10, 0.9, 1.1, b["rng"], b["tok"], b["out"], b["step"],
                                b["pos"], b["lens"], ctr, True)
        assert torch.equal(nb, nxt)
    for k in a:
        assert torch.equal(a[k], b[k]), k
