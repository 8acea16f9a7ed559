"""Vectorised forward sampling of evidence rows (host-side synthetic-input generator).

Equivalent in distribution to pgmpy's BayesianModelSampling.forward_sample
(pgmpy/sampling/Sampling.py:30-): ancestral sampling in topological order,
each variable drawn from its CPT column selected by the sampled parent states.
Used by bench.py to build the seeded synthetic evidence batches of SURVEY.md
§8(d) C3/C5; not part of the accelerated path (and it does not reproduce
pgmpy's RNG stream, so the rows differ from pgmpy's for the same seed).
"""
import networkx as nx
import numpy as np


def forward_sample_codes(model, n, seed=42, order=None):
    """[n_nodes, n] uint8 state codes, rows = nodes in `order` (default sorted(model.nodes()))."""
    rng = np.random.default_rng(seed)
    nodes = sorted(model.nodes()) if order is None else list(order)
    idx = {v: i for i, v in enumerate(nodes)}
    codes = np.empty((len(nodes), n), dtype=np.uint8)
    for v in nx.topological_sort(model):
        cpd = model.get_cpds(v)
        card = int(cpd.cardinality[0])
        table = np.asarray(cpd._values_readonly(), dtype=np.float64).reshape(card, -1)  # (card, prod parent cards)
        parents = list(cpd.variables[1:])
        col = np.zeros(n, dtype=np.int32)
        for p, pc in zip(parents, cpd.cardinality[1:]):
            col *= int(pc)
            col += codes[idx[p]]
        cdf = np.cumsum(table, axis=0)  # (card, cols)
        cdf /= cdf[-1:, :]
        u = rng.random(n)
        c = np.zeros(n, dtype=np.uint8)
        for k in range(card - 1):  # state = number of cdf entries below u (inverse CDF)
            c += u > np.take(cdf[k], col)
        codes[idx[v]] = c
    return codes, nodes


def codes_to_frame(model, codes, nodes, columns=None):
    import pandas as pd

    states = model.states
    columns = nodes if columns is None else columns
    pos = {v: i for i, v in enumerate(nodes)}
    return pd.DataFrame({c: np.asarray(states[c], dtype=object)[codes[pos[c]]] for c in columns})


def leaf_findings_codes(model, n, per_row=4, seed=7):
    """The C4 evidence of SURVEY.md §8(d): every leaf of `model` is an evidence column, and each row
    observes `per_row` of them (chosen per row by a seeded generator) at a forward-sampled state; the
    others are 255 (unobserved).  Returns (codes [n_leaves, n] uint8, leaves, sampled codes, nodes).
    bench.py's C4 line and its parity test build their batch through this one function."""
    leaves = sorted(v for v in model.nodes() if model.out_degree(v) == 0)
    codes, nodes = forward_sample_codes(model, n, seed=seed)
    rng = np.random.default_rng(seed)
    ev = np.full((len(leaves), n), 255, dtype=np.uint8)
    rows = [nodes.index(v) for v in leaves]
    for r in range(n):
        for j in rng.choice(len(leaves), size=per_row, replace=False):
            ev[j, r] = codes[rows[j], r]
    return ev, leaves, codes, nodes
