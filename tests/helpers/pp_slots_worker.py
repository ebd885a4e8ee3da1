"""torchrun target of tests/test_serve_pipeline_cpu.py::test_continuous_batching_over_pipeline:
rank 0's ServingEngine drives continuous batching over a gloo pipeline (parallel.pp_slots).  A
long greedy request starts; once it is decoding, a short one is submitted.  Writes both answers
and the order in which they completed to argv[1].

    pp_slots_worker.py OUT MODEL [STAGES_SEEN]"""
import argparse
import json
import sys
import time

from edgellm.cli.serve import _launch, build_pipeline_engine
from edgellm.engine import SamplingParams


def main():
    out_path, model = sys.argv[1], sys.argv[2]
    args = argparse.Namespace(model=model, precision="fp32", quant="none", device="cpu", base_model_path=None,
                              max_batch=4, max_seq=128, kv_dtype="bf16", static_batches=False)
    launch = _launch(args)
    engine = build_pipeline_engine(args, launch)          # ranks > 0 serve until the driver stops them
    assert engine.continuous, "the pipeline engine serves with continuous batching"
    order = []
    greedy = dict(temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1, do_sample=False)
    long_ids, short_ids = [5, 9, 13, 2], [7, 3]
    f_long = engine.submit(long_ids, SamplingParams(max_new_tokens=48, **greedy))
    f_long.add_done_callback(lambda f: order.append("long"))
    t0 = time.time()
    while engine.stats["decode_steps"] < 4 and time.time() - t0 < 120:
        time.sleep(0.002)
    steps_at_submit = engine.stats["decode_steps"]
    f_short = engine.submit(short_ids, SamplingParams(max_new_tokens=3, **greedy))
    f_short.add_done_callback(lambda f: order.append("short"))
    r_short, r_long = f_short.result(timeout=300), f_long.result(timeout=300)
    metrics = engine.metrics()
    engine.close()                                         # also releases rank 1 (shutdown)
    json.dump({"long": [long_ids, 48, r_long["tokens"]], "short": [short_ids, 3, r_short["tokens"]],
               "order": order, "steps_at_submit": steps_at_submit, "metrics": metrics}, open(out_path, "w"))


if __name__ == "__main__":
    main()
