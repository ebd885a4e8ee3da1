"""edgellm — an MI355X-native distributed-edge LLM inference runtime.

Capabilities mirror the reference project ``parthabp55/LLM-for-Distributed-Egde-Devices``
(see SURVEY.md): single-model and multi-agent-ensemble generation with the
reference's prompts, sampling and metrics, INT8 quantised inference, a
layer-partitioned pipeline across GPUs ("edge devices") and the gRPC/REST
demo services.  The compute path is PyTorch-ROCm plus hand-written CDNA4 HIP
kernels (``edgellm.ops``); GPUs talk over RCCL point-to-point (``edgellm.parallel``).

Import as ``import edgellm`` (the repo-root ``edgellm.py`` maps the hyphenated
directory name onto this package).
"""

__version__ = "0.1.0"

__all__ = ["__version__"]
