"""Vocab-sharded sampler kernels on the GPU (sampler.hip edge_sample_shard / edge_sample_merge):
phase 1 over each shard of a row with global ids, phase 2 over the concatenated candidate lists,
must draw exactly the token the unsplit fused sampler draws from the whole row (greedy, full-vocab
sampling, top-k + top-p, repetition penalty; bf16 and fp32 logits; 256-row batches whose unsplit
sampler takes the whole-row form).  top-k stays below the 128-candidate chunk lists: at k = 128
exact ties at the cut can overflow a list, where both the split and the unsplit sampler truncate —
each at its own chunk boundaries."""
import pytest
import torch

from edgellm import ops
from edgellm.parallel.vocab_head import shard_bounds

pytestmark = pytest.mark.gpu

CFGS = [(0.7, 50, 0.9, 1.1, True), (1.0, 0, 1.0, 1.3, True), (0.7, 20, 1.0, 1.2, False), (0.8, 7, 0.5, 1.1, True),
        (0.7, 100, 0.95, 1.1, True)]


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("B,V", [(5, 32000), (256, 32000), (3, 50257), (4, 128256)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_shard_merge_equals_fused_sampler(cuda, cfg, P, B, V, dt):
    T, k, p, pen, ds = cfg
    g = torch.Generator(device=cuda).manual_seed(B * 7 + P)
    logits = (torch.randn(B, V, device=cuda, generator=g) * 3).to(dt)
    seen = (torch.rand(B, V, device=cuda, generator=g) < 0.05).to(torch.uint8)
    rng = torch.tensor([77, 5], dtype=torch.int32, device=cuda)
    ref = ops.sample(logits, seen.clone(), T, k, p, pen, rng.clone(), ds)
    b = shard_bounds(V, P)
    shards = [ops.sample_shard(logits[:, b[r]:b[r + 1]].contiguous(), seen[:, b[r]:b[r + 1]].contiguous(), T, k, p,
                               pen, rng, b[r], V, ds) for r in range(P)]
    got = ops.sample_merge(shards, V, T, k, p, rng, ds)
    assert torch.equal(got, ref)
    assert torch.equal(rng.cpu(), torch.tensor([77, 5], dtype=torch.int32))     # neither phase advances rng


def test_shard_candidate_shapes_match_kernel(cuda):
    rng = torch.tensor([1, 0], dtype=torch.int32, device=cuda)
    for mode, (T, k, p) in [(2, (0.7, 50, 0.9)), (1, (0.7, 0, 1.0)), (0, (0.0, 0, 1.0))]:
        lg = torch.randn(8, 4032, device=cuda).bfloat16()
        c = ops.sample_shard(lg, None, T, k, p, 1.0, rng, 4032, 32000, T > 0)
        shapes = ops.shard_candidate_shapes(8, 4032, 32000, mode, cuda)
        assert [(tuple(x.shape), x.dtype) for x in c] == [(tuple(s), d) for s, d in shapes]
