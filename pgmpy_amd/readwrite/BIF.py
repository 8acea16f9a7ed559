"""Minimal BIF reader (mirrors pgmpy/readwrite/BIF.py:34-419 semantics).

The reference parses with pyparsing (7.8 s for munin); this is a single-pass
regex tokenizer with the same model semantics:
  * nodes in file order, edges parent -> child from each `probability` header;
  * a row block `(s_p1, ..., s_pk) v_1, ..., v_card;` fills column
    index(product(states of parents)) of the (card, prod parent cards) table
    (BIF.py:281-307);
  * a `table` / `default` block is reshaped to (card, size // card) (BIF.py:287-293);
  * CPDs are added sorted by variable name (BIF.py:383-404), state names as str.
"""
import gzip
import re
from itertools import product

import numpy as np

_VAR_RE = re.compile(r"variable\s+([^\s{]+)\s*\{(.*?)\n\}", re.S)
_STATES_RE = re.compile(r"type\s+discrete\s*\[\s*(\d+)\s*\]\s*\{(.*?)\}", re.S)
_PROB_RE = re.compile(r"probability\s*\(\s*([^)]*?)\s*\)\s*\{(.*?)\n\}", re.S)
_NET_RE = re.compile(r"network\s+([^\s{]+)\s*\{")


class BIFReader:
    def __init__(self, path=None, string=None):
        if string is None:
            opener = gzip.open if str(path).endswith(".gz") else open
            with opener(path, "rt") as f:
                string = f.read()
        self.network = string
        m = _NET_RE.search(string)
        self.network_name = m.group(1) if m else "unknown"
        self.variable_names = []
        self.variable_states = {}
        for name, body in _VAR_RE.findall(string):
            sm = _STATES_RE.search(body)
            if sm is None:
                raise ValueError(f"variable {name}: only discrete variables are supported")
            states = [s.strip() for s in sm.group(2).split(",") if s.strip()]
            if len(states) != int(sm.group(1)):
                raise ValueError(f"variable {name}: declared {sm.group(1)} states, found {len(states)}")
            self.variable_names.append(name)
            self.variable_states[name] = states
        self.variable_parents = {}
        self.variable_cpds = {}
        for header, body in _PROB_RE.findall(string):
            parts = [p.strip() for p in re.split(r"[|,]", header) if p.strip()]
            var, parents = parts[0], parts[1:]
            self.variable_parents[var] = parents
            self.variable_cpds[var] = self._values(var, parents, body)
        self.variable_edges = [[p, v] for v in self.variable_parents for p in self.variable_parents[v]]

    def _values(self, var, parents, body):
        card = len(self.variable_states[var])
        lines = [ln.strip() for ln in body.strip().split(";") if ln.strip()]
        if lines and re.match(r"^(table|default)\b", lines[0]):
            nums = []
            for ln in lines:
                ln = re.sub(r"^(table|default)\b", "", ln)
                nums.extend(float(x) for x in ln.replace(",", " ").split())
            arr = np.array(nums, dtype=np.float64)
            return arr.reshape((card, arr.size // card))
        ncols = int(np.prod([len(self.variable_states[p]) for p in parents])) if parents else 1
        arr = np.zeros((card, ncols))
        rows = {}
        for ln in lines:
            m = re.match(r"^\((.*?)\)\s*(.*)$", ln, re.S)
            if not m:
                continue
            states = tuple(s.strip() for s in m.group(1).split(","))
            rows[states] = [float(x) for x in m.group(2).replace(",", " ").split()]
        for index, comb in enumerate(product(*[self.variable_states[p] for p in parents])):
            arr[:, index] = rows[comb]
        return arr

    def get_model(self, state_name_type=str):
        from ..factors.discrete import TabularCPD
        from ..models import DiscreteBayesianNetwork

        model = DiscreteBayesianNetwork()
        model.add_nodes_from(self.variable_names)
        model.add_edges_from(self.variable_edges)
        model.name = self.network_name
        cpds = []
        for var in sorted(self.variable_cpds):
            sn = {p: list(map(state_name_type, self.variable_states[p])) for p in self.variable_parents[var]}
            sn[var] = list(map(state_name_type, self.variable_states[var]))
            cpds.append(TabularCPD(var, len(self.variable_states[var]), self.variable_cpds[var],
                                   evidence=self.variable_parents[var],
                                   evidence_card=[len(self.variable_states[p]) for p in self.variable_parents[var]],
                                   state_names=sn))
        model.add_cpds(*cpds)
        return model
