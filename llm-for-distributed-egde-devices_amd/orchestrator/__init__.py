from .ensemble import Agent, EnsembleResult, Orchestrator, RefineMerge, VoteMerge
from .prompts import QA_TEMPLATE, REFINE_TEMPLATE, qa_prompt, refine_prompt

__all__ = ["Agent", "EnsembleResult", "Orchestrator", "RefineMerge", "VoteMerge", "QA_TEMPLATE", "REFINE_TEMPLATE",
           "qa_prompt", "refine_prompt"]
