"""Prompt templates and decoding conventions of the reference ensemble."""
from __future__ import annotations

# QA agent prompt (combine_model_fp_updated.py:87-91; Llama_bf16_updated.py:70-74)
QA_TEMPLATE = (
    "You are a helpful assistant. Provide a detailed and informative answer to the following question. "
    "Ensure the answer is at least 50 words long and includes relevant factual details and commonly expected terms.\n\n"
    "Question: {question}\nAnswer:"
)
# CPU-edge variant without "...and commonly expected terms" (Code/C-DAC Server/try.py:239-243)
QA_TEMPLATE_CPU = (
    "You are a helpful assistant. Provide a detailed and informative answer to the following question. "
    "Ensure the answer is at least 50 words long and includes relevant factual details.\n\n"
    "Question: {question}\nAnswer:"
)
# Refiner prompt (combine_model_fp_updated.py:114-122).  NOTE: the reference inserts the gold
# answer as "Reference (optional)" — this inflates the ensemble's scores (SURVEY §6 caveat 2);
# ``include_reference=False`` removes the leak.
REFINE_TEMPLATE = (
    "You are an expert AI assistant. Combine the best information from the two responses below into one clear, "
    "informative answer. The final answer should be at least 50 words long, avoid vague phrases, and include factual "
    "terms or named entities that improve keyword overlap with the reference answer if available.\n\n"
    "Response 1:\n{ans1}\n\n"
    "Response 2:\n{ans2}\n\n"
    "Reference (optional):\n{reference}\n\n"
    "Final refined response:"
)
# N-agent generalisation of the refiner prompt
REFINE_TEMPLATE_N = (
    "You are an expert AI assistant. Combine the best information from the responses below into one clear, "
    "informative answer. The final answer should be at least 50 words long, avoid vague phrases, and include factual "
    "terms or named entities that improve keyword overlap with the reference answer if available.\n\n"
    "{responses}"
    "Reference (optional):\n{reference}\n\n"
    "Final refined response:"
)


def qa_prompt(question: str, cpu_variant: bool = False) -> str:
    return (QA_TEMPLATE_CPU if cpu_variant else QA_TEMPLATE).format(question=question.strip())


def refine_prompt(answers, reference=None, include_reference: bool = True) -> str:
    ref = (reference if reference else "N/A") if include_reference else "N/A"
    if len(answers) == 2:
        return REFINE_TEMPLATE.format(ans1=answers[0], ans2=answers[1], reference=ref)
    body = "".join(f"Response {i + 1}:\n{a}\n\n" for i, a in enumerate(answers))
    return REFINE_TEMPLATE_N.format(responses=body, reference=ref)
