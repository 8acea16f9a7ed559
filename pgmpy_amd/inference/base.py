"""Inference base: model check, factor index, BN pruning (mirror of pgmpy/inference/base.py:19-312)."""
from collections import defaultdict
from itertools import chain

import networkx as nx
import numpy as np

from ..factors.discrete import DiscreteFactor, TabularCPD
from ..models import DiscreteBayesianNetwork, JunctionTree
from .dsep import prune


def _fast_bn(nodes, edges, cpds):
    """A DiscreteBayesianNetwork from a known-acyclic sub-structure (skips per-edge cycle checks)."""
    bn = DiscreteBayesianNetwork()
    nx.DiGraph.add_nodes_from(bn, nodes)
    nx.DiGraph.add_edges_from(bn, edges)
    bn._bump()
    for cpd in cpds:
        bn.cpds.append(cpd)
        bn._cpd_index[cpd.variable] = cpd
    return bn


def prune_structure(model, variables, evidence_vars):
    """Nodes kept by d-separation + ancestral pruning (inference/base.py:154-197), on the
    integer-indexed DAG (pgmpy_amd.inference.dsep.prune).

    Returns (kept_nodes in model order, evidence vars kept)."""
    return prune(model, list(variables), list(evidence_vars))


class Inference(object):
    def __init__(self, model):
        self.model = model
        model.check_model()
        if isinstance(self.model, JunctionTree):
            self.variables = set(chain(*self.model.nodes()))
        else:
            self.variables = self.model.nodes()

    def _initialize_structures(self):
        # inference/base.py:88-152
        if isinstance(self.model, JunctionTree):
            self.variables = set(chain(*self.model.nodes()))
        else:
            self.variables = self.model.nodes()
        self.cardinality = {}
        self.factors = defaultdict(list)
        if isinstance(self.model, DiscreteBayesianNetwork):
            self.state_names_map = {}
            for node in self.model.nodes():
                cpd = self.model.get_cpds(node)
                if isinstance(cpd, TabularCPD):
                    self.cardinality[node] = cpd.variable_card
                    cpd = cpd.to_factor()
                for var in cpd.scope():
                    self.factors[var].append(cpd)
                self.state_names_map.update(cpd.no_to_name)
        else:
            self.cardinality = self.model.get_cardinality()
            for factor in self.model.get_factors():
                for var in factor.variables:
                    self.factors[var].append(factor)

    def _prune_bayesian_model(self, variables, evidence):
        """d-separation + ancestral pruning; CPDs losing parents are summed over them and
        renormalised on the device (TabularCPD.marginalize) (inference/base.py:154-212)."""
        evidence = {} if evidence is None else evidence
        kept, ev = prune_structure(self.model, variables, list(evidence.keys()))
        evidence = {var: state for var, state in evidence.items() if var in ev}
        kept_set = set(kept)
        cpds = []
        for var in kept:
            cpd = self.model.get_cpds(var)
            scope_diff = set(cpd.scope()) - kept_set
            cpds.append(cpd if not scope_diff else cpd.marginalize(scope_diff, inplace=False))
        edges = [(u, v) for u, v in self.model.edges() if u in kept_set and v in kept_set]
        return _fast_bn(kept, edges, cpds), evidence

    def _check_virtual_evidence(self, virtual_evidence):
        # inference/base.py:214-254
        for cpd in virtual_evidence:
            if not isinstance(cpd, (TabularCPD, DiscreteFactor)):
                raise ValueError(
                    f"Virtual evidence should be an instance of TabularCPD or DiscreteFactor. Got: {type(cpd)}")
            if isinstance(cpd, DiscreteFactor) and len(cpd.variables) > 1:
                raise ValueError(f"If cpd is an instance of DiscreteFactor, it should be defined on a single "
                                 f"variable. Got: {cpd}")
            var = cpd.variables[0]
            if var not in self.model.nodes():
                raise ValueError("Evidence provided for variable which is not in the model")
            elif len(cpd.variables) > 1:
                raise ValueError("Virtual evidence should be defined on individual variables. "
                                 "Maybe you are looking for soft evidence.")
            elif self.model.get_cardinality(var) != cpd.get_cardinality([var])[var]:
                raise ValueError("The number of states/cardinality for the evidence should be same as the number "
                                 "of states/cardinality of the variable in the model")

    def _virtual_evidence(self, virtual_evidence):
        """Add a binary child '__var' per virtual evidence (inference/base.py:256-299)."""
        self._check_virtual_evidence(virtual_evidence)
        bn = self.model.copy()
        for cpd in virtual_evidence:
            var = cpd.variables[0]
            new_var = "__" + var
            bn.add_edge(var, new_var)
            v = np.asarray(cpd.values).reshape(-1)
            values = np.vstack((v, 1 - v))
            new_cpd = TabularCPD(variable=new_var, variable_card=2, values=values, evidence=[var],
                                 evidence_card=[self.model.get_cardinality(var)],
                                 state_names={new_var: [0, 1], var: cpd.state_names[var]})
            bn.add_cpds(new_cpd)
        self.__init__(bn)

    @staticmethod
    def _get_virtual_evidence_var_list(virtual_evidence):
        return [cpd.variables[0] for cpd in virtual_evidence]
