from .base import Inference
from .ExactInference import BeliefPropagation, VariableElimination

__all__ = ["Inference", "VariableElimination", "BeliefPropagation"]
