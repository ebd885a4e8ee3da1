from .linear import CPUDynamicLinear, LLMInt8Linear, W8A8Linear, quantize_weight_per_channel
from .smoothquant import (QUANT_MODES, collect_act_absmax, is_graph_safe, quantize_head, quantize_model,
                          smooth_model_, synthetic_calibration)
from .checkpoint import load_quantized, save_quantized

__all__ = ["W8A8Linear", "LLMInt8Linear", "CPUDynamicLinear", "quantize_weight_per_channel", "QUANT_MODES",
           "collect_act_absmax", "is_graph_safe", "quantize_head", "quantize_model", "smooth_model_", "synthetic_calibration",
           "load_quantized", "save_quantized"]
