"""Concurrent generators on one GPU (engine.generate.co_generate — ensemble agents sharing a
device): each generator decodes on its own HIP stream with its own graphs, interleaved from one
host thread; tokens must equal each generator run alone (greedy and seeded sampling), with EOS
exits at different steps."""
import pytest
import torch

from edgellm.engine import Generator, SamplingParams
from edgellm.engine.generate import co_generate
from edgellm.models import build_model, tiny
from edgellm.quant import quantize_model

pytestmark = pytest.mark.gpu


def test_co_generate_matches_solo(cuda):
    cfgs = [tiny("llama", hidden_size=256, num_heads=4, num_kv_heads=2, intermediate_size=512, num_layers=2),
            tiny("gpt_neox", num_layers=3), tiny("llama2", hidden_size=256, num_heads=2, num_kv_heads=2,
                                                   intermediate_size=512, num_layers=2)]
    models = [build_model(cfgs[0], device=cuda, seed=1), build_model(cfgs[1], device=cuda, seed=2),
              quantize_model(build_model(cfgs[2], device=cuda, seed=3), "w8a8")]
    g = torch.Generator().manual_seed(0)
    prompts = [[torch.randint(0, c.vocab_size, (n,), generator=g).tolist() for n in (9, 9, 5)] for c in cfgs]
    sps = [SamplingParams(max_new_tokens=40, do_sample=False, repetition_penalty=1.1),
           SamplingParams(max_new_tokens=33, temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1),
           SamplingParams(max_new_tokens=40, temperature=0.8, top_k=20, top_p=0.95)]
    solo = [Generator(m, max_batch=3, max_seq=64).generate(p, sp, seed=5 + i)
            for i, (m, p, sp) in enumerate(zip(models, prompts, sps))]
    eos = [solo[0].tokens[0][10], None, None]          # first job exits early on its row 0 token
    solo[0] = Generator(models[0], max_batch=3, max_seq=64).generate(prompts[0], sps[0], seed=5, eos_token_id=eos[0])
    gens = [Generator(m, max_batch=3, max_seq=64) for m in models]
    jobs = [(gen, p, sp, 5 + i, e) for i, (gen, p, sp, e) in enumerate(zip(gens, prompts, sps, eos))]
    got = co_generate(jobs)
    for a, b in zip(got, solo):
        assert a.tokens == b.tokens
    assert any(gen._graphs for gen in gens)             # decode ran graph-replayed


def test_continuous_batching_gpu_matches_solo(cuda):
    """SlotDecoder on the GPU (graph-captured masked decode step, W8A8): requests admitted while
    others decode, slots reused after release; greedy tokens equal each request run alone."""
    from edgellm.engine.continuous import SlotDecoder
    cfg = tiny("llama2", hidden_size=256, num_heads=2, num_kv_heads=2, intermediate_size=512, num_layers=2)
    m = quantize_model(build_model(cfg, device=cuda, seed=3), "w8a8")
    g = torch.Generator().manual_seed(1)
    reqs = [(torch.randint(0, cfg.vocab_size, (n,), generator=g).tolist(), k)
            for n, k in ((7, 20), (3, 9), (12, 15), (5, 30), (9, 4), (2, 11))]
    sp = SamplingParams(max_new_tokens=64, do_sample=False, repetition_penalty=1.1)
    dec = SlotDecoder(Generator(m, max_batch=3, max_seq=96), sp)
    got, queue = {}, list(enumerate(reqs))
    while queue or dec.busy():
        while queue and dec.can_admit(len(queue[0][1][0]), queue[0][1][1]):
            i, (ids, k) = queue.pop(0)
            dec.admit(ids, k, None, tag=i)
        dec.step(3)
        for tag, res in dec.poll():
            got[tag] = res.tokens[0]
    assert dec.use_graphs and dec._graphs
    for i, (ids, k) in enumerate(reqs):
        solo = Generator(m, max_batch=1, max_seq=96).generate([ids], SamplingParams(
            max_new_tokens=k, do_sample=False, repetition_penalty=1.1)).tokens[0]
        assert got[i] == solo, i
