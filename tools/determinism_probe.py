#!/usr/bin/env python
"""Run-to-run determinism of the unsplit tiny-model generation the pipeline GPU tests compare
against (tests/test_pipeline_gpu.py::_reference): the same prompts and seeds three times; any
difference means a kernel on that path is not deterministic."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from test_pipeline_gpu import _reference  # noqa: E402

for quant in ("none", "w8a8"):
    for do_sample in (False, True):
        runs = [_reference("llama", quant, 2, 4, 9, 12, do_sample) for _ in range(3)]
        same = all(r == runs[0] for r in runs[1:])
        bad = sorted({i for r in runs[1:] for i, (x, y) in enumerate(zip(r, runs[0])) if x != y})
        print(f"quant={quant} sample={do_sample}: deterministic={same} rows_differing={bad}", flush=True)
