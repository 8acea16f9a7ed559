"""TabularCPD (mirror of pgmpy/factors/discrete/CPD.py:117-596).

A CPT P(X | U1..Uk) stored as a DiscreteFactor over [X, U1..Uk] (flat C-order,
CPD.py:180-182).  normalize / marginalize / reduce renormalise columns; the
column sums and the division run on the device (pgm_contract).
"""
import logging
import numbers

import numpy as np

from ... import engine as E
from .DiscreteFactor import DiscreteFactor

logger = logging.getLogger("pgmpy")


class TabularCPD(DiscreteFactor):
    def __init__(self, variable, variable_card, values, evidence=None, evidence_card=None, state_names={}):
        # CPD.py:117-182
        self.variable = variable
        self.variable_card = None
        variables = [variable]
        if not isinstance(variable_card, numbers.Integral):
            raise TypeError("Event cardinality must be an integer")
        self.variable_card = variable_card
        cardinality = [variable_card]
        if evidence_card is not None:
            if isinstance(evidence_card, numbers.Real):
                raise TypeError("Evidence card must be a list of numbers")
            cardinality.extend(evidence_card)
        if evidence is not None:
            if isinstance(evidence, str):
                raise TypeError("Evidence must be list, tuple or array of strings.")
            if evidence_card is None:
                raise ValueError("Evidence card must be provided if Evidence is provided!")
            variables.extend(evidence)
            if not len(evidence_card) == len(evidence):
                raise ValueError("Length of evidence_card doesn't match length of evidence")
        values_casted = np.array(values, dtype=np.float64)
        if values_casted.ndim != 2:
            raise TypeError("Values must be a 2D list/array")
        expected = (variable_card, 1) if evidence is None else (variable_card, int(np.prod(evidence_card)))
        if values_casted.shape != expected:
            raise ValueError(f"values must be of shape {expected}. Got shape: {values_casted.shape}")
        if not isinstance(state_names, dict):
            raise ValueError(f"state_names must be of type dict. Got {type(state_names)}")
        super(TabularCPD, self).__init__(variables, cardinality, values_casted.flatten(), state_names=state_names)

    def __repr__(self):
        var_str = f"<TabularCPD representing P({self.variable}:{self.variable_card}"
        evidence = self.variables[1:]
        evidence_card = self.cardinality[1:]
        ev = (" | " + ", ".join([f"{v}:{c}" for v, c in zip(evidence, evidence_card)])) if evidence else ""
        return var_str + ev + f") at {hex(id(self))}>"

    def get_values(self):
        # CPD.py:198-223 (a view of values: editing it edits the CPD, so the values are exposed)
        return self._shape2d(self.values)

    def _shape2d(self, v):
        if self.variable in self.variables:
            return v.reshape(tuple([self.cardinality[0], int(np.prod(self.cardinality[1:]))]))
        return v.reshape(tuple([int(np.prod(self.cardinality)), 1]))

    def get_evidence(self):
        return self.variables[:0:-1]

    def copy(self):
        evidence = self.variables[1:] if len(self.variables) > 1 else None
        evidence_card = self.cardinality[1:] if len(self.variables) > 1 else None
        return TabularCPD(self.variable, self.variable_card, np.array(self._shape2d(self._values_readonly())), evidence, evidence_card,
                          state_names=self.state_names.copy())

    def normalize(self, inplace=True):
        """Column-normalise the CPT (CPD.py:449-481) on the device."""
        cpd = self if inplace else self.copy()
        A = cpd._d()
        labels = list(range(A.dim()))
        if A.dim() == 0:
            return None if inplace else cpd
        cols = E.contract(A, labels, None, None, labels[1:], reduce="sum", combine="copy")
        out = E.contract(A, labels, cols, labels[1:], labels, combine="div_raw")
        cpd._set_d(out)
        if not inplace:
            return cpd

    def marginalize(self, variables, inplace=True):
        # CPD.py:483-524
        if self.variable in variables:
            raise ValueError("Marginalization not allowed on the variable on which CPD is defined")
        cpd = self if inplace else self.copy()
        DiscreteFactor.marginalize(cpd, variables)
        cpd.normalize()
        if not inplace:
            return cpd

    def reduce(self, values, inplace=True, show_warnings=True):
        # CPD.py:526-567
        if self.variable in (value[0] for value in values):
            raise ValueError("Reduce not allowed on the variable on which CPD is defined")
        cpd = self if inplace else self.copy()
        DiscreteFactor.reduce(cpd, values, show_warnings=show_warnings)
        cpd.normalize()
        if not inplace:
            return cpd

    def to_factor(self):
        # CPD.py:569-596
        f = DiscreteFactor.__new__(DiscreteFactor)
        f.variables = self.variables.copy()
        f.cardinality = self.cardinality.copy()
        f._host = None
        f._dev = None
        if self._dev is not None:
            f._dev = E.copy(self._dev)
        else:
            f._host = np.array(self._host)
        f.state_names = self.state_names.copy()
        f.name_to_no = self.name_to_no.copy()
        f.no_to_name = self.no_to_name.copy()
        return f

    def reorder_parents(self, new_order, inplace=True):
        """The CPT with its parents (evidence) in `new_order` (CPD.py:598-727): the values transposed
        on the device (one strided copy, pgm_contract).  inplace=True re-initialises the CPD over
        [variable] + new_order and returns get_values() — as the reference does through
        DiscreteFactor.__init__ without state names, so the state names become 0..card-1;
        inplace=False returns the reordered 2-D values and leaves the CPD as it was."""
        if (len(self.variables) <= 1 or (set(new_order) - set(self.variables))
                or (set(self.variables[1:]) - set(new_order))):
            raise ValueError("New order either has missing or extra arguments")
        if list(new_order) == list(self.variables[1:]):
            logger.warning("Same ordering provided as current")
            return self.get_values()
        card = dict(zip(self.variables, (int(c) for c in self.cardinality)))
        A = self._d()
        labels = list(self.variables)
        out_labels = [self.variables[0]] + list(new_order)
        moved = E.contract(A, labels, None, None, out_labels, combine="copy")
        if inplace:
            cardinality = [self.variable_card] + [card[v] for v in new_order]
            DiscreteFactor.__init__(self, out_labels, cardinality, moved)
            return self.get_values()
        return E.to_host(moved).reshape(self.cardinality[0], int(np.prod([card[v] for v in new_order])))

    def to_dataframe(self):
        """The CPT as a DataFrame (CPD.py:336-410): one row per combination of the parents' states
        (a MultiIndex named after them, parents in the CPD's order), one column per state of the
        variable (columns named after it), each row a conditional distribution."""
        import pandas as pd

        idx = pd.MultiIndex.from_product([self.state_names[v] for v in self.variables], names=self.variables)
        flat = pd.DataFrame({"probability": np.asarray(self._values_readonly()).ravel()}, index=idx)
        return flat["probability"].unstack(self.variable)

    def is_valid_cpd(self):
        v = self._shape2d(self._values_readonly())  # internal read: does not expose the values
        return bool(np.allclose(v.sum(axis=0), np.ones(v.shape[1]), atol=0.01))
