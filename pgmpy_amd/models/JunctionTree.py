"""JunctionTree (mirror of pgmpy/models/JunctionTree.py:8-152 + ClusterGraph.py:130-365).

An undirected tree whose nodes are cliques (tuples of variables) with one
clique potential (DiscreteFactor) per clique.  The BP engine
(pgmpy_amd.inference.ExactInference.BeliefPropagation) calibrates it on the
device.
"""
import copy as _copy

import networkx as nx
import numpy as np


class JunctionTree(nx.Graph):
    def __init__(self, ebunch=None):
        super().__init__()
        self.factors = []
        if ebunch:
            self.add_edges_from(ebunch)

    def add_node(self, node, **kwargs):
        if not isinstance(node, (list, set, tuple)):
            raise TypeError("Node can only be a list, set or tuple of nodes forming a clique")
        super().add_node(tuple(node), **kwargs)

    def add_nodes_from(self, nodes, **kwargs):
        for n in nodes:
            self.add_node(n, **kwargs)

    def add_edge(self, u, v, **kwargs):
        u, v = tuple(u), tuple(v)
        if u in self.nodes() and v in self.nodes() and nx.has_path(self, u, v):
            raise ValueError(f"Addition of edge between {str(u)} and {str(v)} forms a cycle breaking the "
                             "properties of Junction Tree")
        super().add_edge(u, v, **kwargs)

    def add_edges_from(self, ebunch, **kwargs):
        for u, v in ebunch:
            self.add_edge(u, v, **kwargs)

    def add_factors(self, *factors):
        # ClusterGraph.py:130-164
        for factor in factors:
            if set(factor.scope()) not in [set(n) for n in self.nodes()]:
                raise ValueError("Factors defined on clusters of variable notpresent in model")
            self.factors.append(factor)

    def get_factors(self, node=None):
        # ClusterGraph.py:166-198
        if node is None:
            return self.factors
        if set(node) not in [set(n) for n in self.nodes()]:
            raise ValueError("Node not present in Cluster Graph")
        return next(filter(lambda x: set(x.scope()) == set(node), self.factors))

    def remove_factors(self, *factors):
        for f in factors:
            self.factors.remove(f)

    def get_cardinality(self, node=None):
        if node:
            for factor in self.factors:
                for variable, card in zip(factor.scope(), factor.cardinality):
                    if node == variable:
                        return card
        card = {}
        for factor in self.factors:
            for variable, c in zip(factor.scope(), factor.cardinality):
                card[variable] = c
        return card

    @property
    def states(self):
        return {node: states for phi in self.factors for node, states in phi.state_names.items()}

    def check_model(self):
        # JunctionTree.py:118-137, ClusterGraph.py:329-365
        if len(self.nodes()) > 1 and not nx.is_connected(self):
            raise ValueError("The Junction Tree defined is not fully connected.")
        for clique in self.nodes():
            factors = list(filter(lambda x: set(x.scope()) == set(clique), self.factors))
            if not factors:
                raise ValueError("Factors for all the cliques or clusters not defined.")
        cardinalities = self.get_cardinality()
        if len(set((x for clique in self.nodes() for x in clique))) != len(cardinalities):
            raise ValueError("Factors for all the variables not defined.")
        for factor in self.factors:
            for variable, cardinality in zip(factor.scope(), factor.cardinality):
                if cardinalities[variable] != cardinality:
                    raise ValueError(f"Cardinality of variable {variable} not matching among factors")
        return True

    def copy(self):
        jt = JunctionTree(self.edges())
        jt.add_nodes_from(self.nodes())
        if self.factors:
            jt.add_factors(*[f.copy() for f in self.factors])
        return jt

    def __deepcopy__(self, memo):
        return self.copy()
