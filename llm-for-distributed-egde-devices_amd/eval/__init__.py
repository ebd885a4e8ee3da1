from .text_metrics import corpus_bleu, evaluate_bleu, evaluate_rouge, mean_rouge, rouge_scores, rouge_tokenize
from .metrics import (METRIC_KEYS, EfficiencyMeter, Embedder, MetricSuite, ProgressLog, Results, bertscore_f1, confidence_score,
                      cosine_similarity)

__all__ = ["corpus_bleu", "evaluate_bleu", "evaluate_rouge", "mean_rouge", "rouge_scores", "rouge_tokenize",
           "METRIC_KEYS", "EfficiencyMeter", "Embedder", "MetricSuite", "ProgressLog", "Results", "bertscore_f1", "confidence_score",
           "cosine_similarity"]
