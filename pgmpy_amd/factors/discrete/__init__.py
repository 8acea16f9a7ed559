from .DiscreteFactor import DiscreteFactor
from .CPD import TabularCPD

__all__ = ["DiscreteFactor", "TabularCPD"]
