"""Host side of the batch-1 persistent decode engine (engine/b1_engine.py <-> ops/csrc/b1_engine.hip).

The kernel walks each wave's weight stream in a fixed order (for every layer: qkv, o, gate_up, down;
within a projection the CU's units, unit-major, then the wave's k-blocks) and reads lane l's 16 bytes
of a fragment as W[col 4 (l >> 2)][k 16 (l & 3) ..].  These tests replay that walk in Python against
the layout the host builds, for uneven unit splits (units not divisible by the CU count)."""
import pytest
import torch

from edgellm.engine.b1_engine import _phase_units, stream_layout, unit_split


def _walk(ws, fmax, mats, H, F, NQ, QH, G):
    """Yield (c, w, fragment index, expected 1 KiB) in the kernel's consumption order."""
    uq, uh, uf = unit_split(NQ // 16, G), unit_split(H // 16, G), unit_split(F // 8, G)
    kbq, kbo, kbd = H // 256, QH // 256, F // 256
    for c in range(G):
        for w in range(4):
            g = 0
            for mat in mats:
                for ph, (q, sp, kbw) in enumerate(zip(mat, (uq, uh, uf, uh), (kbq, kbo, kbq, kbd))):
                    units = _phase_units(q, glu=ph == 2)                   # [NU, 16, K]
                    for u in range(int(sp[c]), int(sp[c + 1])):
                        for kb in range(w * kbw, (w + 1) * kbw):
                            blk = units[u, :, kb * 64:(kb + 1) * 64]          # [16 cols, 64 k]
                            # lane = 4 col + ksub: W[col][16 ksub .. +16]
                            exp = blk.reshape(16, 4, 16).reshape(-1)
                            yield c, w, g, exp
                            g += 1


@pytest.mark.parametrize("G", [4, 5, 7])
def test_stream_layout_matches_kernel_walk(G):
    torch.manual_seed(0)
    H, F, Hq, Hkv, HD, L = 256, 512, 2, 1, 128, 2
    NQ, QH = (Hq + 2 * Hkv) * HD, Hq * HD
    r = lambda *s: torch.randint(-127, 128, s, dtype=torch.int8)          # noqa: E731
    mats = [(r(NQ, H), r(H, QH), r(2 * F, H), r(H, F)) for _ in range(L)]
    ws, fmax = stream_layout(mats, H, F, NQ, QH, G)
    assert ws.shape == (G, 4, fmax, 1024)
    n = 0
    for c, w, g, exp in _walk(ws, fmax, mats, H, F, NQ, QH, G):
        assert g < fmax
        assert torch.equal(ws[c, w, g], exp), (c, w, g)
        n += 1
    # every fragment of every projection appears exactly once across the streams
    assert n == L * (NQ * H + H * QH + 2 * F * H + H * F) // 1024


def test_gate_up_units_pair_gate_and_up_rows():
    F, K = 32, 256
    q = torch.arange(2 * F, dtype=torch.int32)[:, None].expand(2 * F, K).to(torch.int8)
    u = _phase_units(q, glu=True)
    assert u.shape == (F // 8, 16, K)
    for j in range(F // 8):
        assert u[j, :8, 0].tolist() == list(range(8 * j, 8 * j + 8))            # gate rows
        assert u[j, 8:, 0].tolist() == list(range(F + 8 * j, F + 8 * j + 8))   # up rows


def test_unit_split_even():
    s = unit_split(1376, 256)
    n = (s[1:] - s[:-1])
    assert int(s[-1]) == 1376 and int(n.min()) == 5 and int(n.max()) == 6
    assert int(unit_split(768, 256).diff().max()) == 3
