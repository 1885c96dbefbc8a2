"""MI355X-native top-N scoring path of hyunlord/hnm_recommendation.

Embedding lookup -> all-items scoring (NeuralCF / LightGCN / Wide&Deep / MF) -> top-K,
as hand-written gfx950 HIP kernels behind the C ABI in include/hnm.h (libhnm_mi355x.so),
exposed through modules that mirror the reference's `src/models` surface.
"""
from .evaluation import RecommendationMetrics
from .models import LightGCN, MatrixFactorization, NeuralCF, UserHistory, WideDeep

__all__ = ["NeuralCF", "LightGCN", "WideDeep", "MatrixFactorization", "RecommendationMetrics",
           "UserHistory"]
