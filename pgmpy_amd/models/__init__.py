from .ClusterGraph import ClusterGraph
from .DiscreteBayesianNetwork import DiscreteBayesianNetwork
from .DiscreteMarkovNetwork import DiscreteMarkovNetwork
from .FactorGraph import FactorGraph
from .JunctionTree import JunctionTree

# pgmpy < 1.0 names
BayesianNetwork = DiscreteBayesianNetwork
MarkovNetwork = DiscreteMarkovNetwork

__all__ = ["ClusterGraph", "DiscreteBayesianNetwork", "BayesianNetwork", "DiscreteMarkovNetwork", "MarkovNetwork",
           "FactorGraph", "JunctionTree"]
