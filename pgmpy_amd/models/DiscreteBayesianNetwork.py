"""DiscreteBayesianNetwork (the hot path's container and data-parallel caller).

Mirrors the parts of pgmpy/models/DiscreteBayesianNetwork.py and
pgmpy/base/DAG.py the hot path touches: CPD bookkeeping (add_cpds/get_cpds
L243-353), check_model (L451-508), moralize (DAG.py:449), d-separation
(active_trail_nodes DAG.py:864-950, _get_ancestors_of L952-990,
get_ancestral_graph L1163-1186), to_junction_tree (L539-594) and the
data-parallel callers predict / predict_probability (L731-989).

predict / predict_probability do not loop over rows in Python: rows are
grouped by evidence pattern (which columns are observed), each pattern is
compiled once into a device plan (pgmpy_amd.inference.plan) and every row of
the pattern runs in one fused kernel launch.
"""
import logging
from collections import defaultdict

import networkx as nx
import numpy as np

from .. import engine as E
from ..factors.discrete import TabularCPD

logger = logging.getLogger("pgmpy")


class DiscreteBayesianNetwork(nx.DiGraph):
    def __init__(self, ebunch=None, latents=set()):
        super().__init__()
        self.cpds = []
        self._cpd_index = {}
        self.cardinalities = defaultdict(int)
        self.latents = set(latents)
        self._epoch = 0  # bumped on every structural / CPD change (plan caches key on it)
        if ebunch:
            self.add_edges_from(ebunch)

    # ------------------------------------------------------------------ structure
    def add_edge(self, u, v, **kwargs):
        if u == v:
            raise ValueError("Self loops are not allowed.")
        if u in self.nodes() and v in self.nodes() and nx.has_path(self, v, u):
            raise ValueError(f"Loops are not allowed. Adding the edge from ({u}->{v}) forms a loop.")
        super().add_edge(u, v, **kwargs)
        self._bump()

    def _bump(self):
        self.__dict__["_epoch"] = self.__dict__.get("_epoch", 0) + 1

    def add_node(self, node, **kwargs):
        super().add_node(node, **kwargs)
        self._bump()

    def add_nodes_from(self, nodes, **kwargs):
        super().add_nodes_from(nodes, **kwargs)
        self._bump()

    def remove_edge(self, u, v):
        super().remove_edge(u, v)
        self._bump()

    def remove_edges_from(self, ebunch):
        super().remove_edges_from(ebunch)
        self._bump()

    def remove_node(self, n):
        super().remove_node(n)
        self._bump()

    def remove_nodes_from(self, nodes):
        super().remove_nodes_from(nodes)
        self._bump()

    def add_edges_from(self, ebunch, **kwargs):
        for e in ebunch:
            self.add_edge(*e[:2], **kwargs)

    def get_parents(self, node):
        return list(self.predecessors(node))

    def get_children(self, node):
        return list(self.successors(node))

    def moralize(self):
        """Moral graph (DAG.py:449-470): drop directions, marry co-parents."""
        g = nx.Graph()
        g.add_nodes_from(self.nodes())
        g.add_edges_from(self.to_undirected().edges())
        for node in self.nodes():
            ps = list(self.predecessors(node))
            for i in range(len(ps)):
                for j in range(i + 1, len(ps)):
                    g.add_edge(ps[i], ps[j])
        return g

    # ------------------------------------------------------------------ CPDs
    def add_cpds(self, *cpds):
        # DiscreteBayesianNetwork.py:243-283
        for cpd in cpds:
            if not isinstance(cpd, TabularCPD):
                raise ValueError("Only TabularCPD can be added.")
            if set(cpd.scope()) - set(cpd.scope()).intersection(set(self.nodes())):
                raise ValueError("CPD defined on variable not in the model", cpd)
            if cpd.variable in self._cpd_index:
                logger.warning(f"Replacing existing CPD for {cpd.variable}")
                for i, c in enumerate(self.cpds):
                    if c.variable == cpd.variable:
                        self.cpds[i] = cpd
                        break
            else:
                self.cpds.append(cpd)
            self._cpd_index[cpd.variable] = cpd
        self._bump()

    def get_cpds(self, node=None):
        if node is not None:
            if node not in self.nodes():
                raise ValueError("Node not present in the Directed Graph")
            return self._cpd_index.get(node)
        return self.cpds

    def remove_cpds(self, *cpds):
        for cpd in cpds:
            if isinstance(cpd, (str, int)):
                cpd = self.get_cpds(cpd)
            self.cpds.remove(cpd)
            self._cpd_index.pop(cpd.variable, None)
        self._bump()

    def get_cardinality(self, node=None):
        if node is not None:
            return self.get_cpds(node).cardinality[0]
        return defaultdict(int, {cpd.variable: cpd.cardinality[0] for cpd in self.cpds})

    @property
    def states(self):
        return {var: self.get_cpds(var).state_names[var] for var in self.nodes()}

    def check_model(self):
        # DiscreteBayesianNetwork.py:451-508
        for node in self.nodes():
            cpd = self.get_cpds(node=node)
            if cpd is None:
                raise ValueError(f"No CPD associated with {node}")
            evidence = cpd.get_evidence()
            if set(evidence) != set(self.get_parents(node)):
                raise ValueError(f"CPD associated with {node} doesn't have proper parents associated with it.")
            if len(set(cpd.variables) - set(cpd.state_names.keys())) > 0:
                raise ValueError(f"CPD for {node} doesn't have state names defined for all the variables.")
            if not cpd.is_valid_cpd():
                raise ValueError(f"Sum or integral of conditional probabilities for node {node} is not equal to 1.")
        for node in self.nodes():
            cpd = self.get_cpds(node=node)
            for index, par in enumerate(cpd.variables[1:]):
                parent_cpd = self.get_cpds(par)
                if parent_cpd.cardinality[0] != cpd.cardinality[1 + index]:
                    raise ValueError(f"The cardinality of {par} doesn't match in it's child nodes.")
                if parent_cpd.state_names[par] != cpd.state_names[par]:
                    raise ValueError(f"The state names of {par} doesn't match in it's child nodes.")
        return True

    def copy(self):
        m = DiscreteBayesianNetwork(latents=self.latents)
        m.add_nodes_from(self.nodes())
        m.add_edges_from(self.edges())
        if self.cpds:
            m.add_cpds(*[cpd.copy() for cpd in self.cpds])
        return m

    @E.serialized
    def get_state_probability(self, states):
        """P(states) for a full or partial assignment {variable: state name}
        (DiscreteBayesianNetwork.py:991-1041; same checks, same ValueError messages).

        The reference sums the product of every CPD over every combination of the unassigned variables
        (itertools.product: exponential in their number — alarm with 6 of 37 unassigned is ~500
        combinations, munin is out of reach).  Here only the assigned variables' ancestors take part
        (every other CPD sums to 1 over its own variable: barren), each CPD is sliced at the assigned
        states as a strided view of its device values, and what is left is ONE planned contraction to
        a scalar on the device (inference.contraction.contract_factors, the greedy-path machinery of
        VariableElimination.query); CPDs fully inside the assignment contribute one host value each."""
        self.check_model()
        for var, state in states.items():
            if var not in self.nodes():
                raise ValueError(f"{var} not in the model.")
            if state not in self.states[var]:
                raise ValueError(f"State: {state} not define for {var}")
        if not states:
            return 1.0
        from ..inference.contraction import contract_factors

        anc = self._get_ancestors_of(list(states))
        host = 1.0
        ops = []
        for node in self.nodes():
            if node not in anc:
                continue
            cpd = self.get_cpds(node)
            idx = {v: cpd.name_to_no[v][states[v]] for v in cpd.variables if v in states}
            rest = [v for v in cpd.variables if v not in idx]
            if not rest:
                host *= float(cpd._values_readonly()[tuple(idx[v] for v in cpd.variables)])
                continue
            t = cpd._d()
            if idx:
                t = t[tuple(idx[v] if v in idx else slice(None) for v in cpd.variables)]
            ops.append((t, rest))
        if not ops:
            return host
        return host * float(E.to_host(contract_factors(ops, [])).reshape(-1)[0])

    # ------------------------------------------------------------------ d-separation (DAG.py)
    def _get_ancestors_of(self, nodes):
        if not isinstance(nodes, (list, tuple)):
            nodes = [nodes]
        for node in nodes:
            if node not in self.nodes():
                raise ValueError(f"Node {node} not in graph")
        anc = set()
        for node in nodes:
            anc.update(nx.ancestors(self, node))
        anc.update(nodes)
        return anc

    def active_trail_nodes(self, variables, observed=None, include_latents=False):
        """{variable: nodes reachable from it by an active trail given `observed`} (DAG.py:864-950).

        Computed on the integer-indexed DAG (pgmpy_amd.inference.dsep, Bayes-ball)."""
        from ..inference.dsep import active_trails

        if observed is None or (not isinstance(observed, (str, int)) and len(observed) == 0):
            observed = []
        elif isinstance(observed, (str, int)) or not hasattr(observed, "__iter__"):
            observed = [observed]
        starts = variables if isinstance(variables, (list, tuple, set)) else [variables]
        return active_trails(self, list(starts), list(observed), include_latents=include_latents)

    def get_ancestral_graph(self, nodes):
        anc = self._get_ancestors_of(list(nodes))
        g = DiscreteBayesianNetwork()
        g.add_nodes_from([n for n in self.nodes() if n in anc])
        g.add_edges_from([(u, v) for u, v in self.edges() if u in anc and v in anc])
        return g

    # ------------------------------------------------------------------ junction tree
    def to_markov_model(self):
        """The moral graph with one potential per CPD (DiscreteBayesianNetwork.py:510-537)."""
        from .DiscreteMarkovNetwork import DiscreteMarkovNetwork

        moral = self.moralize()
        mm = DiscreteMarkovNetwork(moral.edges())
        mm.add_nodes_from(moral.nodes())
        mm.add_factors(*[cpd.to_factor() for cpd in self.cpds])
        return mm

    def to_junction_tree(self):
        """Junction tree with clique potentials = product of the CPDs assigned to each clique.

        The reference triangulates with heuristic H6 (DiscreteMarkovNetwork.py:324-518),
        which builds a 75-variable clique on pathfinder (ValueError) and a 95.5M-state
        clique on alarm (SURVEY.md headline 4).  This uses a proper min-fill elimination
        (pgmpy_amd.inference.EliminationOrder.min_fill_cliques); the calibrated marginals
        are the same distribution (BP is exact on any junction tree)."""
        from ..inference.EliminationOrder import junction_tree_from_model

        return junction_tree_from_model(self)

    # ------------------------------------------------------------------ data-parallel callers
    @E.serialized
    def predict(self, data, algo=None, stochastic=False, n_jobs=-1, seed=None, **kwargs):
        """MAP of the missing variables per row (DiscreteBayesianNetwork.py:731-910).

        Rows are grouped by evidence pattern; each pattern is one compiled device plan
        (fused one-lane-per-row kernel).  The output frame matches the reference:
        columns data.columns + missing variables, rows in index order, state names."""
        from ..inference.batch import column_checks, predict_frame

        column_checks(self, data)  # the reference's ValueErrors (cached per columns object)
        if algo is not None:
            from ..inference import Inference

            if not (isinstance(algo, type) and issubclass(algo, Inference)):
                raise TypeError(f"Algorithm should be a valid pgmpy inference method. Got {type(algo)} instead.")
        if stochastic:
            from ..inference.batch import predict_stochastic_frame

            return predict_stochastic_frame(self, data, seed=seed)
        return predict_frame(self, data)

    @E.serialized
    def predict_probability(self, data):
        """Per-row marginals of every missing variable (DiscreteBayesianNetwork.py:912-989)."""
        from ..inference.batch import column_checks, predict_probability_frame

        column_checks(self, data)  # the reference's ValueErrors (cached per columns object)
        return predict_probability_frame(self, data)
