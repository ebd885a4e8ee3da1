"""torchrun target of tests/test_serve_pipeline_cpu.py::test_continuous_batching_4_ranks_staggered:
rank 0's ServingEngine serves 16 staggered greedy requests over a 4-stage gloo pipeline
(parallel.pp_slots: batched ragged admission, on-device token budgets).  The last request is
short and submitted while long ones decode; writes every answer, the completion order and the
engine metrics to argv[1].

    pp_slots_load_worker.py OUT MODEL [VOCAB_SPLIT on|off]"""
import argparse
import json
import sys
import time

from edgellm.cli.serve import _launch, build_pipeline_engine
from edgellm.engine import SamplingParams


def main():
    out_path, model = sys.argv[1], sys.argv[2]
    vs = sys.argv[3] if len(sys.argv) > 3 else "off"
    args = argparse.Namespace(model=model, precision="fp32", quant="none", device="cpu", base_model_path=None,
                              max_batch=16, max_seq=128, kv_dtype="bf16", static_batches=False,
                              pp_vocab_split=vs, partition="units")   # tiny:llama: 2 layers = 4 half-layer units
    launch = _launch(args)
    engine = build_pipeline_engine(args, launch)          # ranks > 0 serve until the driver stops them
    greedy = dict(temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1, do_sample=False)
    reqs = []
    for i in range(15):                                   # prompt lengths 2-9, 20-40 new tokens
        ids = [(7 * i + 3 * j) % 250 + 3 for j in range(2 + i % 8)]
        reqs.append((f"r{i}", ids, 20 + (i * 7) % 21))
    reqs.append(("short", [11, 4, 9], 2))
    order, futs = [], {}
    t0 = time.time()
    for n, (key, ids, mx) in enumerate(reqs):
        if key == "short":                                # once the long ones are decoding
            while engine.stats["decode_steps"] < 6 and time.time() - t0 < 120:
                time.sleep(0.002)
        f = engine.submit(ids, SamplingParams(max_new_tokens=mx, **greedy))
        f.add_done_callback(lambda f, k=key: order.append(k))
        futs[key] = f
        if n % 4 == 3:
            time.sleep(0.01)                              # staggered arrivals
    res = {k: f.result(timeout=600)["tokens"] for k, f in futs.items()}
    metrics = engine.metrics()
    vs_session = bool(getattr(engine.gen._slot_sess, "vs", False))
    engine.close()                                        # also releases ranks 1-3 (shutdown)
    json.dump({"requests": [[k, ids, mx] for k, ids, mx in reqs], "tokens": res, "order": order,
               "metrics": metrics, "vs_session": vs_session}, open(out_path, "w"))


if __name__ == "__main__":
    main()
