"""Register-spill guard for the kernels that count their own LDS-DMA with inline
``s_waitcnt vmcnt(N)``: a spill's scratch loads / stores join the same counter, so a spilling
ring kernel waits for the wrong operations and reads LDS before its DMA landed (round 2: a 10-wave
decode kernel spilled 236 B/lane and produced non-deterministic slices).  Cross-compiles for
gfx950 on the CPU (tools/kernel_resources.py) and requires zero scratch in every kernel of the
files that hold such rings."""
import os
import shutil
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "llm-for-distributed-egde-devices_amd", "ops", "csrc")
RING_FILES = ["gemm_i8.hip", "gemm_i8_prefill.hip", "attn_prefill.hip", "sampler.hip", "b1_engine.hip"]   # every file with an inline vmcnt


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="no hipcc")
def test_counted_vmcnt_kernels_do_not_spill():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kernel_resources import resources
    with ThreadPoolExecutor(len(RING_FILES)) as ex:
        reports = dict(zip(RING_FILES, ex.map(lambda f: resources(os.path.join(CSRC, f)), RING_FILES)))
    assert all(reports.values()), "no kernel resource remarks (compile failed?)"
    spills = {f"{f}:{k}": v.get("ScratchSize", 0) for f, rep in reports.items() for k, v in rep.items()
              if v.get("ScratchSize", 0) > 0}
    assert not spills, spills
