"""REST front-end (FastAPI): the reference's time endpoint plus generation and metrics.

``GET /``          -> ``{"current_time": "YYYY-MM-DD HH:MM:SS"}``  (rest_api.py:9-11, port 8000)
``POST /generate`` -> run the attached engine (edgellm.serve.server.ServingEngine)
``GET /health``, ``GET /metrics`` (JSON counters: requests, tokens, p50/p99 step latency)
"""
# no ``from __future__ import annotations``: FastAPI must resolve the locally defined request model
from typing import List, Optional

from .time_service import now_string


def make_app(engine=None):
    from fastapi import FastAPI, HTTPException
    from pydantic import BaseModel

    import contextlib

    @contextlib.asynccontextmanager
    async def lifespan(_app):
        yield
        # server shutdown (Ctrl-C on uvicorn): drain the engine and release a pipeline's worker ranks
        if engine is not None and hasattr(engine, "close"):
            engine.close()

    app = FastAPI(title="edgellm", lifespan=lifespan)

    class GenerateRequest(BaseModel):
        prompt: Optional[str] = None
        prompt_ids: Optional[List[int]] = None
        max_new_tokens: int = 64
        temperature: float = 0.7
        top_k: int = 50
        top_p: float = 0.9
        repetition_penalty: float = 1.1
        do_sample: bool = True
        seed: int = 0

    @app.get("/")
    def get_time():
        return {"current_time": now_string()}

    @app.get("/health")
    def health():
        return {"status": "ok", "engine": engine is not None}

    @app.get("/metrics")
    def metrics():
        return engine.metrics() if engine is not None else {}

    @app.post("/generate")
    def generate(req: GenerateRequest):
        if engine is None:
            raise HTTPException(503, "no engine attached")
        return engine.generate_request(req.model_dump() if hasattr(req, "model_dump") else req.dict())

    return app


def serve(host: str = "0.0.0.0", port: int = 8000, engine=None):  # pragma: no cover - CLI
    import uvicorn
    uvicorn.run(make_app(engine), host=host, port=port)
