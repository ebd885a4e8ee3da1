from .configs import ModelConfig, PRESETS, get_config, tiny, from_hf_config
from .decoder import AttnCtx, DecoderLM, build_model, init_random_, global_named_parameters
from .layers import Linear, Norm, QAct

__all__ = ["ModelConfig", "PRESETS", "get_config", "tiny", "from_hf_config", "AttnCtx", "DecoderLM",
           "build_model", "init_random_", "global_named_parameters", "Linear", "Norm", "QAct"]
