from .DiscreteBayesianNetwork import DiscreteBayesianNetwork
from .FactorGraph import FactorGraph
from .JunctionTree import JunctionTree

# pgmpy < 1.0 name
BayesianNetwork = DiscreteBayesianNetwork

__all__ = ["DiscreteBayesianNetwork", "BayesianNetwork", "FactorGraph", "JunctionTree"]
