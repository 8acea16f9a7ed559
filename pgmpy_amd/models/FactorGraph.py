"""FactorGraph (mirror of pgmpy/models/FactorGraph.py): a bipartite undirected graph of variable
nodes and DiscreteFactor nodes, the model BeliefPropagationWithMessagePassing runs on.

Same constructor and methods as the reference (FactorGraph.py:17-518) for what the message-passing
inference needs: add_edge (no self loops), add_factors (optionally replacing a factor over the same
scope), remove_factors, get_cardinality, check_model (bipartite, every factor node holds a factor,
cardinalities agree), get_variable_nodes, get_factor_nodes, get_factors, get_partition_function,
copy, get_point_mass_message and get_uniform_message.  Factor values stay device-resident; the
partition function is one device contraction.
"""
from collections import defaultdict

import networkx as nx
import numpy as np
from networkx.algorithms import bipartite

from ..factors.discrete import DiscreteFactor


class FactorGraph(nx.Graph):
    def __init__(self, ebunch=None):
        # FactorGraph.py:65-69
        super().__init__()
        if ebunch:
            self.add_edges_from(ebunch)
        self.factors = []

    def add_edge(self, u, v, **kwargs):
        # FactorGraph.py:71-95
        if u == v:
            raise ValueError("Self loops are not allowed")
        kwargs.setdefault("weight", 0)
        super().add_edge(u, v, **kwargs)

    def add_factors(self, *factors, replace=False):
        # FactorGraph.py:97-137
        for factor in factors:
            if set(factor.variables) - set(factor.variables).intersection(set(self.nodes())):
                raise ValueError("Factors defined on variable not in the model", factor.__repr__())
            if replace:
                for fa in list(self.factors):
                    if set(factor.variables) == set(fa.variables):
                        neighbors = list(self.neighbors(fa)) if fa in self else []
                        self.remove_factors(fa)
                        self.add_node(factor)
                        self.add_edges_from([(factor, neigh) for neigh in neighbors])
            self.factors.append(factor)

    def remove_factors(self, *factors):
        # FactorGraph.py:139-157
        for factor in factors:
            self.factors.remove(factor)
            if factor in self.nodes:
                self.remove_node(factor)

    def get_cardinality(self, node=None):
        # FactorGraph.py:159-203
        if node:
            for factor in self.factors:
                for variable, cardinality in zip(factor.scope(), factor.cardinality):
                    if node == variable:
                        return cardinality
            return None
        cardinalities = defaultdict(int)
        for factor in self.factors:
            for variable, cardinality in zip(factor.scope(), factor.cardinality):
                cardinalities[variable] = cardinality
        return cardinalities

    def check_model(self):
        # FactorGraph.py:205-247
        variable_nodes = set(x for factor in self.factors for x in factor.scope())
        factor_nodes = set(self.nodes()) - variable_nodes
        if not all(isinstance(f, DiscreteFactor) for f in factor_nodes):
            raise ValueError("Factors not associated for all the random variables")
        if not bipartite.is_bipartite(self) or not bipartite.is_bipartite_node_set(self, variable_nodes):
            raise ValueError("Edges can only be between variables and factors")
        if len(factor_nodes) != len(self.factors):
            raise ValueError("Factors not associated with all the factor nodes.")
        cardinalities = self.get_cardinality()
        if len(variable_nodes) != len(cardinalities):
            raise ValueError("Factors for all the variables not defined")
        for factor in self.factors:
            for variable, cardinality in zip(factor.scope(), factor.cardinality):
                if cardinalities[variable] != cardinality:
                    raise ValueError(f"Cardinality of variable {variable} not matching among factors")
        return True

    def get_variable_nodes(self):
        # FactorGraph.py:249-273
        self.check_model()
        return list(set(x for factor in self.factors for x in factor.scope()))

    def get_factor_nodes(self):
        # FactorGraph.py:275-301
        self.check_model()
        variable_nodes = self.get_variable_nodes()
        return list(set(self.nodes()) - set(variable_nodes))

    def to_markov_model(self):
        # FactorGraph.py:303-336: each factor's scope becomes a clique of the Markov network
        from itertools import combinations

        from .DiscreteMarkovNetwork import DiscreteMarkovNetwork

        mm = DiscreteMarkovNetwork()
        variable_nodes = self.get_variable_nodes()
        if len(set(self.nodes()) - set(variable_nodes)) != len(self.factors):
            raise ValueError("Factors not associated with all the factor nodes.")
        mm.add_nodes_from(variable_nodes)
        for factor in self.factors:
            mm.add_edges_from(combinations(factor.scope(), 2))
            mm.add_factors(factor)
        return mm

    def to_junction_tree(self):
        # FactorGraph.py:338-361
        return self.to_markov_model().to_junction_tree()

    def get_factors(self, node=None):
        # FactorGraph.py:363-397
        if node is None:
            return self.factors
        if node not in self.get_factor_nodes():
            raise ValueError("Factors are not associated with the corresponding node.")
        return [f for f in self.factors if set(f.scope()) == set(self.neighbors(node))][0]

    def get_partition_function(self):
        # FactorGraph.py:399-431: sum of the product of all factors (one device contraction)
        from ..engine import to_host
        from ..inference.contraction import contract_factors

        variables = set(self.get_variable_nodes())
        if set(v for f in self.factors for v in f.scope()) != variables:
            raise ValueError("DiscreteFactor for all the random variables not defined.")
        total = contract_factors([(f._d(), list(f.variables)) for f in self.factors], [])
        return float(to_host(total))

    def copy(self):
        # FactorGraph.py:433-466
        copy = FactorGraph()
        copy.add_nodes_from(self.nodes())
        copy.add_edges_from(self.edges())
        copy.add_factors(*[f.copy() for f in self.factors])
        return copy

    def get_point_mass_message(self, variable, observation):
        # FactorGraph.py:468-495
        message = np.zeros(self.get_cardinality(variable))
        message[observation] = 1
        return message

    def get_uniform_message(self, variable):
        # FactorGraph.py:497-518
        card = self.get_cardinality(variable)
        return np.ones(card) / card
