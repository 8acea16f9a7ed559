from .base import Inference
from .ExactInference import BeliefPropagation, BeliefPropagationWithMessagePassing, VariableElimination

__all__ = ["Inference", "VariableElimination", "BeliefPropagation", "BeliefPropagationWithMessagePassing"]
