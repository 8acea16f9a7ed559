"""JunctionTree (mirror of pgmpy/models/JunctionTree.py:8-152).

A ClusterGraph (pgmpy_amd.models.ClusterGraph) that stays a tree: add_edge refuses an edge that
would close a cycle (JunctionTree.py:55-78) and check_model additionally requires connectivity
(L96-114).  One clique potential (DiscreteFactor) per clique; the BP engine
(pgmpy_amd.inference.ExactInference.BeliefPropagation) calibrates it on the device.
"""
import networkx as nx

from .ClusterGraph import ClusterGraph


class JunctionTree(ClusterGraph):
    def add_edge(self, u, v, **kwargs):
        u, v = tuple(u), tuple(v)
        if u in self.nodes() and v in self.nodes() and nx.has_path(self, u, v):
            raise ValueError(f"Addition of edge between {str(u)} and {str(v)} forms a cycle breaking the "
                             "properties of Junction Tree")
        super().add_edge(u, v, **kwargs)

    def check_model(self):
        if len(self.nodes()) > 1 and not nx.is_connected(self):
            raise ValueError("The Junction Tree defined is not fully connected.")
        return super().check_model()

    def copy(self):
        # JunctionTree.py:116-152: edges first, then every node (isolated ones included)
        jt = JunctionTree(self.edges())
        jt.add_nodes_from(self.nodes())
        if self.factors:
            jt.add_factors(*[f.copy() for f in self.factors])
        return jt
