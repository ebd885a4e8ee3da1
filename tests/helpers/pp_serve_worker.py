"""torchrun target of tests/test_serve_pipeline_cpu.py (and the GPU rehearsal in
tests/test_multiproc_gpu.py): the REST engine over a gloo pipeline.  Rank 0 posts POST /generate
requests through a FastAPI TestClient (concurrently, or one after another with ``seq``) and writes
the tokens to argv[1]; the other ranks serve the pipeline commands until the driver stops them.

    pp_serve_worker.py OUT MODEL [DEVICE [PRECISION [MAX_BATCH [seq]]]]"""
import argparse
import json
import sys
import threading

from edgellm.cli.serve import _launch, build_pipeline_engine
from edgellm.parallel.pp_engine import stop_workers


def main():
    out_path, model = sys.argv[1], sys.argv[2]
    device = sys.argv[3] if len(sys.argv) > 3 else "cpu"
    precision = sys.argv[4] if len(sys.argv) > 4 else "fp32"
    max_batch = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    sequential = len(sys.argv) > 6 and sys.argv[6] == "seq"
    args = argparse.Namespace(model=model, precision=precision, quant="none", device=device, base_model_path=None,
                              max_batch=max_batch, max_seq=128, kv_dtype="bf16")
    launch = _launch(args)
    engine = build_pipeline_engine(args, launch)          # ranks > 0 never return
    from fastapi.testclient import TestClient
    from edgellm.serve.rest import make_app
    client = TestClient(make_app(engine))
    reqs = [{"prompt_ids": [1, 2, 3 + i], "max_new_tokens": 5 + (i % 3), "do_sample": False} for i in range(6)]
    res = [None] * len(reqs)

    def post(i):
        r = client.post("/generate", json=reqs[i])
        res[i] = r.json()["tokens"] if r.status_code == 200 else r.text

    if sequential:
        for i in range(len(reqs)):
            post(i)
    else:
        th = [threading.Thread(target=post, args=(i,)) for i in range(len(reqs))]
        for t in th:
            t.start()
        for t in th:
            t.join()
    metrics = client.get("/metrics").json()
    engine.close()
    stop_workers(engine.gen)
    json.dump({"requests": reqs, "tokens": res, "metrics": metrics}, open(out_path, "w"))


if __name__ == "__main__":
    main()
