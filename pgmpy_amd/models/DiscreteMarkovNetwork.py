"""DiscreteMarkovNetwork (mirror of pgmpy/models/DiscreteMarkovNetwork.py:16-882).

An undirected graph of variables with arbitrary non-negative potentials (DiscreteFactor, values on
the device).  VariableElimination and BeliefPropagation accept it exactly as the reference does:
VE contracts the potentials without pruning or normalisation (ExactInference.py:393-402, 434-438),
BP calibrates the junction tree `to_junction_tree()` builds.

Container (L77-286): add_edge refuses self loops, add_factors refuses factors over variables not in
the graph, get_factors(node) lists the factors holding node, get_cardinality / states from the
factors, check_model checks consistent cardinalities, a factor for every variable and that every
factor's scope is a clique of the graph.

Triangulation (L324-518).  The reference scores every node v of the graph formed by the edges
(isolated nodes are not part of it) with
  S(v) = size of the maximal clique holding all neighbours of v once v is eliminated,
  M(v), C(v) = max / sum of the sizes of the maximal cliques holding v and all its neighbours
(size = product of cardinalities), and deletes in the order of the chosen heuristic
H1 S, H2 S/card(v), H3 S-M, H4 S-C, H5 S/M, H6 S/C.  The reference recomputes the scores of the
remaining nodes on the *unchanged* graph in each of its n rounds, so the order is the nodes sorted
by their score; this restatement scores each node once, from its neighbourhood only:
  * in the graph with v's neighbourhood N completed, the only maximal clique holding v and all of
    N is {v} + N, so M = C = card(v) * prod card(N);
  * the maximal cliques holding N after v's removal are N + Q for Q a maximal clique of the
    graph induced on the common neighbours of N (outside N + {v}).
Ties (the reference breaks them by set iteration order, i.e. string hashes) go to the earlier
node in the graph's node order, and so does the choice among several maximal cliques holding N.
Elimination then adds the fill-in edges of each deleted node's current neighbours (L502-507).

to_junction_tree (L520-637): maximal cliques of the triangulated graph, a maximum-weight spanning
tree over |sepset| (networkx minimum_spanning_tree on negated weights, as the reference), each
factor assigned to the first clique containing its scope, clique potential = ones x product of
its factors (built on the device, in the clique's variable order); unused factors raise.
"""
import itertools
from collections import defaultdict

import networkx as nx
import numpy as np


def _size(nodes, card):
    return float(np.prod([card[x] for x in nodes])) if nodes else 1.0


class DiscreteMarkovNetwork(nx.Graph):
    def __init__(self, ebunch=None, latents=[]):
        super().__init__()
        self.factors = []
        if ebunch:
            self.add_edges_from(ebunch)
        self.latents = latents

    # ------------------------------------------------------------------ structure
    def add_edge(self, u, v, **kwargs):
        if u == v:
            raise ValueError("Self loops are not allowed")
        super().add_edge(u, v, **kwargs)

    def add_edges_from(self, ebunch, **kwargs):
        for e in ebunch:
            self.add_edge(e[0], e[1], **kwargs)

    def is_clique(self, nodes):
        """UndirectedGraph.py:171-208."""
        return all(self.has_edge(a, b) for a, b in itertools.combinations(nodes, 2))

    def is_triangulated(self):
        """UndirectedGraph.py:210-231."""
        return nx.is_chordal(self)

    def markov_blanket(self, node):
        return self.neighbors(node)

    # ------------------------------------------------------------------ potentials
    def add_factors(self, *factors):
        nodes = set(self.nodes())
        for factor in factors:
            if set(factor.variables) - nodes:
                raise ValueError("Factors defined on variable not in the model", factor)
            self.factors.append(factor)

    def get_factors(self, node=None):
        if node:
            if node not in self.nodes():
                raise ValueError("Node not present in the Undirected Graph")
            return [f for f in self.factors if node in f.scope()]
        return self.factors

    def remove_factors(self, *factors):
        for factor in factors:
            self.factors.remove(factor)

    def get_cardinality(self, node=None):
        if node:
            for factor in self.factors:
                for variable, cardinality in zip(factor.scope(), factor.cardinality):
                    if node == variable:
                        return cardinality
            return None
        card = defaultdict(int)
        for factor in self.factors:
            for variable, cardinality in zip(factor.scope(), factor.cardinality):
                card[variable] = cardinality
        return card

    @property
    def states(self):
        return {node: states for phi in self.factors for node, states in phi.state_names.items()}

    def check_model(self):
        cardinalities = self.get_cardinality()
        n_nodes = len(self.nodes())
        for factor in self.factors:
            for variable, cardinality in zip(factor.scope(), factor.cardinality):
                if cardinalities[variable] != cardinality:
                    raise ValueError(f"Cardinality of variable {variable} not matching among factors")
                if n_nodes != len(cardinalities):
                    raise ValueError("Factors for all the variables not defined")
            for a, b in itertools.combinations(factor.variables, 2):
                if not self.has_edge(a, b):
                    raise ValueError("DiscreteFactor inconsistent with the model.")
        return True

    # ------------------------------------------------------------------ conversions
    def to_factor_graph(self):
        """DiscreteMarkovNetwork.py:288-322: one factor node "phi_<scope>" per potential."""
        from .FactorGraph import FactorGraph

        if not self.factors:
            raise ValueError("Factors not associated with the random variables.")
        fg = FactorGraph()
        fg.add_nodes_from(self.nodes())
        for factor in self.factors:
            scope = factor.scope()
            fnode = "phi_" + "_".join(map(str, scope))
            fg.add_edges_from(itertools.product(scope, [fnode]))
            fg.add_factors(factor)
        return fg

    # ------------------------------------------------------------------ triangulation
    def _elimination_scores(self, graph, card):
        """{v: (S, M, C)} for every node of `graph` (see the module docstring)."""
        order = {n: i for i, n in enumerate(graph.nodes())}
        scores = {}
        for v in graph.nodes():
            nbrs = list(graph.neighbors(v))
            m = card[v] * _size(nbrs, card)
            if nbrs:
                common = set.intersection(*[set(graph.neighbors(u)) for u in nbrs]) - set(nbrs) - {v}
                if common:
                    sub = graph.subgraph(common)
                    best = None
                    for q in nx.find_cliques(sub):
                        key = min(order[x] for x in q)
                        if best is None or key < best[0]:
                            best = (key, q)
                    s = _size(nbrs, card) * _size(best[1], card)
                else:
                    s = _size(nbrs, card)
            else:
                s = 1.0
            scores[v] = (s, m, m)
        return scores

    def triangulate(self, heuristic="H6", order=None, inplace=False):
        self.check_model()
        if self.is_triangulated():
            return None if inplace else self
        graph = nx.Graph(self.edges())
        if not order:
            card = self.get_cardinality()
            sc = self._elimination_scores(graph, card)
            key = {
                "H1": lambda v: sc[v][0],
                "H2": lambda v: sc[v][0] / card[v],
                "H3": lambda v: sc[v][0] - sc[v][1],
                "H4": lambda v: sc[v][0] - sc[v][2],
                "H5": lambda v: sc[v][0] / sc[v][1],
            }.get(heuristic, lambda v: sc[v][0] / sc[v][2])
            order = sorted(graph.nodes(), key=key)  # stable: ties keep graph node order
        fill = set()
        for node in order:
            nbrs = list(graph.neighbors(node))
            for a, b in itertools.combinations(nbrs, 2):
                graph.add_edge(a, b)
                fill.add((a, b))
            graph.remove_node(node)
        if inplace:
            for a, b in fill:
                self.add_edge(a, b)
            return self
        tri = DiscreteMarkovNetwork(self.edges())
        for a, b in fill:
            tri.add_edge(a, b)
        return tri

    def to_junction_tree(self):
        from ..factors import factor_product
        from ..factors.discrete import DiscreteFactor
        from .. import engine as E
        from .JunctionTree import JunctionTree

        all_state_names = {}
        for factor in self.factors:
            all_state_names.update(factor.state_names)
        self.check_model()
        tri = self.triangulate()
        cliques = [tuple(c) for c in nx.find_cliques(tri)]
        jt = JunctionTree()
        if len(cliques) == 1:
            jt.add_node(cliques[0])
        elif len(cliques) >= 2:
            complete = nx.Graph()
            for a, b in itertools.combinations(cliques, 2):
                complete.add_edge(a, b, weight=-len(set(a) & set(b)))
            jt = JunctionTree(nx.minimum_spanning_tree(complete).edges())
        card = self.get_cardinality()
        used = [False] * len(self.factors)
        potentials = []
        for clique in jt.nodes():
            members = []
            for i, factor in enumerate(self.factors):
                if not used[i] and set(factor.scope()).issubset(clique):
                    members.append(factor)
                    used[i] = True
            shape = [int(card[v]) for v in clique]
            ones = E.to_device(np.ones(shape))
            if members:
                prod = factor_product(*members) if len(members) > 1 else members[0]
                vals = E.contract(ones, list(clique), prod._d(), list(prod.variables), list(clique), combine="mul")
            else:
                vals = ones
            potentials.append(DiscreteFactor(
                list(clique), shape, vals,
                state_names={v: all_state_names.get(v, list(range(int(card[v])))) for v in clique}))
        jt.add_factors(*potentials)
        if not all(used):
            raise ValueError("All the factors were not used to create Junction Tree.Extra factors are defined.")
        return jt

    def to_bayesian_model(self):
        """Minimal I-map (DiscreteMarkovNetwork.py:719-798): per connected component, order the
        variables by the junction-tree clique (BFS from its first clique) in which each first
        appears; parents = earlier variables of that clique.  Structure only, as the reference."""
        from .DiscreteBayesianNetwork import DiscreteBayesianNetwork

        final = DiscreteBayesianNetwork()
        for comp in nx.connected_components(self):
            sub = nx.Graph(self.subgraph(comp).edges())
            if not sub.number_of_edges():
                final.add_nodes_from(comp)
                continue
            # the reference triangulates the factor-less component with H6, whose scores are all
            # 0/0 there (no cardinalities), i.e. an arbitrary order; min-degree is used instead
            tri = DiscreteMarkovNetwork(sub.edges()).triangulate(order=sorted(sub.nodes(), key=sub.degree))
            if tri is None:
                final.add_nodes_from(comp)
                continue
            cliques = [tuple(c) for c in nx.find_cliques(tri)]
            tree = nx.Graph()
            tree.add_nodes_from(cliques)
            if len(cliques) > 1:
                complete = nx.Graph()
                for a, b in itertools.combinations(cliques, 2):
                    complete.add_edge(a, b, weight=-len(set(a) & set(b)))
                tree = nx.minimum_spanning_tree(complete)
            root = next(iter(tree.nodes()))
            home, order = {}, []
            for clique in [root] + [e[1] for e in nx.bfs_edges(tree, root)]:
                for v in clique:
                    if v not in home:
                        home[v] = clique
                        order.append(v)
            for i, v in enumerate(order):
                parents = (set(home[v]) - {v}) & set(order[:i])
                final.add_edges_from([(p, v) for p in parents])
            final.add_nodes_from(comp)
        return final

    def get_partition_function(self):
        """Sum over all variables of the product of the potentials (L800-844), one device contraction."""
        from ..engine import to_host
        from ..inference.contraction import contract_factors

        self.check_model()
        if set(v for f in self.factors for v in f.scope()) != set(self.nodes()):
            raise ValueError("DiscreteFactor for all the random variables not defined.")
        total = contract_factors([(f._d(), list(f.variables)) for f in self.factors], [])
        return float(to_host(total))

    def copy(self):
        clone = DiscreteMarkovNetwork(self.edges())
        clone.add_nodes_from(self.nodes())
        if self.factors:
            clone.add_factors(*[f.copy() for f in self.factors])
        return clone
