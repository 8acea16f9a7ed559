"""Elimination-order heuristics and junction-tree construction (host-side plan).

The four greedy heuristics restate pgmpy/inference/EliminationOrder.py:11-166
as written, including its quirks (MinFill counts pairs of DiGraph *successors*
and never adds fill-in edges, L107-116/L160-166) so classic-VE orders match
the reference's.  Orders only change floating-point rounding, never results.

junction_tree_from_model() replaces the reference's H6 triangulation
(pgmpy/models/DiscreteMarkovNetwork.py:324-637), which is infeasible on the
target networks (SURVEY.md headline 4), with a min-fill tree decomposition of
the moral graph; clique potentials are the product of the CPDs assigned to the
first clique holding their scope (the SURVEY.md §8(c) "BP oracle" JT).
"""
from itertools import combinations

import networkx as nx
import numpy as np


class BaseEliminationOrder:
    def __init__(self, model):
        from ..models import DiscreteBayesianNetwork

        if not isinstance(model, DiscreteBayesianNetwork):
            raise ValueError("Model should be a DiscreteBayesianNetwork instance")
        self.bayesian_model = nx.DiGraph(model.edges())
        self.bayesian_model.add_nodes_from(model.nodes())
        self.moralized_model = model.moralize()
        self.card = {n: int(model.get_cardinality(n)) for n in model.nodes()}

    def cost(self, node):
        return 0

    def get_elimination_order(self, nodes=None, show_progress=True):
        # EliminationOrder.py:41-105
        if nodes is None:
            nodes = self.bayesian_model.nodes()
        nodes = set(nodes)
        ordering = []
        while nodes:
            scores = {node: self.cost(node) for node in nodes}
            min_score_node = min(scores, key=scores.get)
            ordering.append(min_score_node)
            nodes.remove(min_score_node)
            self.bayesian_model.remove_node(min_score_node)
            self.moralized_model.remove_node(min_score_node)
        return ordering

    def fill_in_edges(self, node):
        return combinations(self.bayesian_model.neighbors(node), 2)


class WeightedMinFill(BaseEliminationOrder):
    def cost(self, node):
        edges = combinations(self.moralized_model.neighbors(node), 2)
        return sum([self.card[a] * self.card[b] for a, b in edges])


class MinNeighbors(BaseEliminationOrder):
    def cost(self, node):
        return len(list(self.moralized_model.neighbors(node)))


class MinWeight(BaseEliminationOrder):
    def cost(self, node):
        return np.prod([self.card[n] for n in self.moralized_model.neighbors(node)])


class MinFill(BaseEliminationOrder):
    def cost(self, node):
        return len(list(self.fill_in_edges(node)))


def min_fill_decomposition(model):
    """(bags, edges): min-fill tree decomposition of the moral graph (sorted-tuple bags)."""
    from networkx.algorithms.approximation import treewidth_min_fill_in

    moral = model.moralize()
    g = nx.Graph(moral.edges())
    g.add_nodes_from(model.nodes())
    _, decomp = treewidth_min_fill_in(g)
    bags = [tuple(sorted(b)) for b in decomp.nodes()]
    edges = [(tuple(sorted(a)), tuple(sorted(b))) for a, b in decomp.edges()]
    return bags, edges


def build_junction_tree(model, bags, edges):
    """JunctionTree over `bags` with potentials = product of assigned CPDs (device ops)."""
    from ..factors import factor_product
    from ..factors.discrete import DiscreteFactor
    from ..models import JunctionTree
    from .. import engine as E

    jt = JunctionTree()
    for b in bags:
        jt.add_node(b)
    for a, b in edges:
        jt.add_edge(a, b)
    assigned = {b: [] for b in bags}
    for node in sorted(model.nodes()):
        cpd = model.get_cpds(node)
        scope = set(cpd.scope())
        for b in bags:
            if scope <= set(b):
                assigned[b].append(cpd.to_factor())
                break
        else:
            raise ValueError(f"no clique covers the scope of {node}")
    card = {n: int(model.get_cardinality(n)) for n in model.nodes()}
    factors = []
    for b in bags:
        sn = {v: model.get_cpds(v).state_names[v] for v in b}
        if assigned[b]:
            pot = factor_product(*assigned[b]) if len(assigned[b]) > 1 else assigned[b][0]
            # broadcast to the full clique in bag order (ones over unassigned variables)
            ones = E.to_device(np.ones([card[v] for v in b]))
            vals = E.contract(ones, list(b), pot._d(), pot.variables, list(b), combine="mul")
        else:
            vals = E.to_device(np.ones([card[v] for v in b]))
        factors.append(DiscreteFactor(list(b), [card[v] for v in b], vals, state_names=sn))
    jt.add_factors(*factors)
    return jt


def junction_tree_from_model(model):
    bags, edges = min_fill_decomposition(model)
    return build_junction_tree(model, bags, edges)
