"""Start the serving front-ends.

    python -m edgellm.cli.serve                                   # TimeService :50051 + REST :8000
    python -m edgellm.cli.serve --model tiny:llama --rest-port 8000     # + POST /generate engine
    python -m edgellm.cli.serve --model gpt2 --stage 6:12 --grpc-port 50052  # a gRPC pipeline stage
    torchrun --nproc-per-node 4 -m edgellm.cli.serve --model llama-2-7b --quant w8a8_smoothquant
                                                                  # engine pipelined over 4 GPUs (RCCL)

TimeService and ``GET /`` are wire-compatible with the reference demo (Code/gRPC/server.py,
rest_api.py); the stage service speaks edgellm.Stage (serve/proto/edgellm_stage.proto).
"""
from __future__ import annotations

import argparse
import threading
from typing import List, Optional

from ..utils.log import get_logger

log = get_logger("serve")


def parse(argv: Optional[List[str]] = None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--grpc-port", type=int, default=50051)
    ap.add_argument("--rest-port", type=int, default=8000)
    ap.add_argument("--no-rest", action="store_true")
    ap.add_argument("--model", default=None, help="attach a generation engine (preset, tiny:<arch> or HF dir)")
    ap.add_argument("--precision", default="bf16", help="bf16 | fp16 | fp32 (GPU: fp16 and bf16 kernels; fp32 and INT8 models run bf16)")
    ap.add_argument("--quant", default="none")
    ap.add_argument("--device", default=None)
    ap.add_argument("--base_model_path", default=None)
    ap.add_argument("--max-batch", type=int, default=8)
    ap.add_argument("--max-seq", type=int, default=2048)
    ap.add_argument("--stage", default=None, help="first:last — serve these layers as a gRPC pipeline stage")
    ap.add_argument("--pp-size", type=int, default=1, help="split the engine's layers over this many GPUs")
    ap.add_argument("--gpus", default=None, help="comma list of GPU ids for the engine (overrides --pp-size)")
    ap.add_argument("--headinfer-heads", type=int, default=None, help="HeadInfer: KV heads per layer kept on the GPU")
    ap.add_argument("--prefill-chunk", type=int, default=4096, help="chunked prefill size (HeadInfer)")
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "int8"])
    ap.add_argument("--partition", default="balanced",
                    help="torchrun pipeline: balanced | units (half-layer bounds) | uniform | '8,8,8,8'")
    ap.add_argument("--pp-lanes", type=int, default=1, help="torchrun pipeline: concurrent micro-batches per stage")
    ap.add_argument("--pp-slack", type=int, default=0, help="torchrun pipeline: extra ticks per stage hop")
    ap.add_argument("--pp-vocab-split", default="on", choices=["on", "off"],
                    help="torchrun pipeline (static batches): LM head split by vocabulary over the stages")
    ap.add_argument("--calib", default="stage", choices=["stage", "full"],
                    help="torchrun + w8a8_smoothquant: per-stage calibration over P2P (stage) or full model")
    ap.add_argument("--static-batches", action="store_true",
                    help="pipeline engine: run each batch to completion (default: continuous batching)")
    return ap.parse_args(argv)


def build(args: argparse.Namespace):
    """Create (started gRPC server, bound port, FastAPI app or None, serving engine or None)."""
    import torch
    import grpc
    from concurrent import futures
    from ..serve.time_service import time_service_handler
    device = args.device or ("cuda:0" if torch.cuda.is_available() else "cpu")
    engine, extra = None, []
    if args.model and args.stage:
        from ..models.registry import load_model
        from ..serve.stage_service import StageServer
        a, b = (int(x) for x in args.stage.split(":"))
        model, _, src = load_model(args.model, args.precision, args.quant, device, base_dir=args.base_model_path,
                                   first=a, last=b)
        extra.append(StageServer(model, max_seq=args.max_seq).handler())
        log.info(f"stage layers [{a}, {b}) of {src}")
    elif args.model and _launch(args) is not None:
        engine = build_pipeline_engine(args, _launch(args))
    elif args.model:
        from ..models.registry import load_model
        from ..parallel.split import agent_devices, split_model
        from ..serve.server import ServingEngine
        from .common import build_generator
        gpus = [int(g) for g in args.gpus.split(",")] if args.gpus else None
        devs = agent_devices(gpus, torch.device(device), args.pp_size)
        model, tok, src = load_model(args.model, args.precision, args.quant, devs[0], base_dir=args.base_model_path)
        if len(devs) > 1:
            model = split_model(model, devs)
        rt = dict(max_seq=args.max_seq, headinfer_heads=args.headinfer_heads, prefill_chunk=args.prefill_chunk,
                  kv_dtype=args.kv_dtype)
        engine = ServingEngine(build_generator(model, rt, max_batch=args.max_batch), tok, args.max_batch)
        log.info(f"generation engine: {src} on {[str(d) for d in devs]}")
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=10),           # server.py:14
                         options=[("grpc.max_receive_message_length", 256 << 20),
                                  ("grpc.max_send_message_length", 256 << 20)])
    server.add_generic_rpc_handlers((time_service_handler(), *extra))
    port = server.add_insecure_port(f"[::]:{args.grpc_port}")
    server.start()
    app = None
    if not args.no_rest:
        from ..serve.rest import make_app
        app = make_app(engine)
    return server, port, app, engine


_LAUNCH = {}


def _launch(args):
    """torchrun (WORLD_SIZE > 1): (rank, world, device) with the process group up, else None."""
    if "v" not in _LAUNCH:
        from .common import pp_launch
        _LAUNCH["v"] = pp_launch({"pp_size": None, "devices": args.device or ""})
    return _LAUNCH["v"]


def build_pipeline_engine(args, launch):
    """Serving over the RCCL pipeline (one process per GPU under torchrun): every rank builds its
    stage (``build_pp_engine``; an INT8 checkpoint directory as ``--model`` is read per stage), rank
    0 wraps its ``PipelineGenerator`` in the ServingEngine; every other rank serves the driver's
    pipeline commands (``serve_workers``) and never returns.  Requests are batched per sampling
    configuration into the pipeline's M micro-batches of b rows.  Default: continuous batching
    (parallel.pp_slots: the M x b rows are slots; a request joins between decode rounds and
    leaves when done); ``--static-batches``: each batch runs to completion across all stages."""
    from ..parallel.pp_engine import serve_workers
    from ..serve.server import ServingEngine
    from .common import build_pp_engine
    rt = dict(max_seq=args.max_seq, kv_dtype=args.kv_dtype, base_model_path=args.base_model_path,
              partition=getattr(args, "partition", "balanced"), pp_lanes=getattr(args, "pp_lanes", 1),
              pp_slack=getattr(args, "pp_slack", 0), calib=getattr(args, "calib", "stage"),
              pp_vocab_split=getattr(args, "pp_vocab_split", "on") == "on")
    eng, tok, src, bounds = build_pp_engine(args.model, args.precision, args.quant, rt, launch, tag=0,
                                            max_batch=args.max_batch)
    if launch[0] != 0:
        serve_workers({0: eng})
        raise SystemExit(0)
    log.info(f"generation engine: {src} pipelined over {launch[1]} ranks at layers {bounds}")
    # continuous batching over the pipeline rows (parallel.pp_slots); --static-batches: run each
    # batch of equal-sampling requests to completion instead
    srv = ServingEngine(eng, tok, args.max_batch, continuous=not getattr(args, "static_batches", False))
    import atexit
    atexit.register(srv.close)             # release the worker ranks however rank 0 exits
    return srv


def main(argv: Optional[List[str]] = None):
    args = parse(argv)
    server, port, app, _ = build(args)
    print(f"gRPC Server running on port {port}...")
    if app is None:
        server.wait_for_termination()
        return
    import uvicorn
    threading.Thread(target=server.wait_for_termination, daemon=True).start()
    uvicorn.run(app, host=args.host, port=args.rest_port)


if __name__ == "__main__":
    main()
