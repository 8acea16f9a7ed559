"""Networks for the oracle, loaded from the reference's own CPT export (ORACLE — test infrastructure only).

tests/golden/networks/<net>_cpts.npz was written by tests/golden/make_golden.py
from the reference's BIFReader (pgmpy/readwrite/BIF.py:361-414) via
get_example_model (pgmpy/utils/utils.py:16-171), so the oracle does not depend
on the product's BIF parser.
"""
import json
import os

import numpy as np

from .factor import OFactor

GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


class ONetwork:
    def __init__(self, nodes, states, parents, cpts):
        self.nodes = list(nodes)
        self.states = states
        self.parents = parents
        self.cpts = cpts  # var -> ndarray shaped (card_var, *card_parents), C-order over [var, *parents]
        self.children = {v: [] for v in self.nodes}
        for v in self.nodes:
            for p in parents[v]:
                self.children[p].append(v)
        self.card = {v: len(states[v]) for v in self.nodes}

    def factor(self, var):
        return OFactor([var] + list(self.parents[var]), self.cpts[var].shape, self.cpts[var])

    def state_no(self, var, name):
        return self.states[var].index(name)


def load_network(name):
    z = np.load(os.path.join(GOLDEN, "networks", f"{name}_cpts.npz"), allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    cpts = {}
    for i, v in enumerate(meta["nodes"]):
        shape = [len(meta["states"][v])] + [len(meta["states"].get(p) or meta["parent_states"][v][p])
                                             for p in meta["parents"][v]]
        cpts[v] = z[f"v{i}"].reshape(shape)
    return ONetwork(meta["nodes"], meta["states"], meta["parents"], cpts)
