from .headinfer import HeadInferKV, heads_for_budget

__all__ = ["HeadInferKV", "heads_for_budget"]
