"""Drop-in mirrors of the reference `src/models` scoring surface (`src/models/__init__.py:3-15`)."""
from .lightgcn import LightGCN
from .matrix_factorization import MatrixFactorization
from .neural_cf import NeuralCF
from .base import UserHistory
from .wide_deep import WideDeep

__all__ = ["NeuralCF", "LightGCN", "WideDeep", "MatrixFactorization", "UserHistory"]
