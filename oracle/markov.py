"""numpy restatement of inference on a DiscreteMarkovNetwork (ORACLE — test infrastructure only).

  query()          ExactInference.py:246-440 for a non-Bayesian model: no pruning, every potential
                   (including those left scalar by the evidence, L393-402) enters the greedy
                   contraction, and the result is NOT normalised (L415-422, L434-438)
  map_query()      ExactInference.py:528-624 / 141-229: argmax (first flat index) of the
                   unnormalised joint of `variables` (all variables when empty)
  max_marginal()   ExactInference.py:459-526: max of the max-product joint over `variables`
  partition()      DiscreteMarkovNetwork.py:800-844
  triangulate()    DiscreteMarkovNetwork.py:324-518, scores straight from the reference's
                   definitions (maximal cliques of the completed neighbourhood graph via networkx),
                   ties broken by graph node order
  jt_cliques()     DiscreteMarkovNetwork.py:520-588 (maximal cliques of the triangulated graph)
  calibrate()      ExactInference.py:770-895 on a junction tree over the given cliques (oracle.bp)
"""
import itertools

import networkx as nx
import numpy as np

from . import bp as OBP
from .factor import OFactor, product_all
from .ve import greedy_contract


def _reduced(factors, evidence):
    out = []
    for f in factors:
        ev = {v: s for v, s in evidence.items() if v in f.vars}
        out.append(f.reduce(ev) if ev else f)
    return out


def query(factors, variables, evidence):
    """Unnormalised sum_{others} prod potentials(evidence), over `variables` in that order."""
    ops = _reduced(factors, evidence)
    scalars = [o for o in ops if not o.vars]
    rest = [o for o in ops if o.vars]
    val = greedy_contract(rest, list(variables)) if rest else np.ones([])
    for s in scalars:
        val = val * float(s.values)
    return val


def joint_all(factors, variables, evidence):
    """The product of all reduced potentials summed to `variables` (all free variables if empty)."""
    ops = _reduced(factors, evidence)
    if not variables:
        j = product_all(ops)
        return j.values, list(j.vars)
    return query(factors, variables, evidence), list(variables)


def map_query(factors, variables, evidence, states):
    j, order = joint_all(factors, variables, evidence)
    idx = int(np.argmax(j))
    out = {}
    for i in reversed(range(len(order))):
        c = j.shape[i]
        out[order[i]] = states[order[i]][idx % c]
        idx //= c
    return out


def max_marginal(factors, variables, evidence):
    ops = _reduced(factors, evidence or {})
    j = product_all(ops)
    keep = list(variables) if variables else list(j.vars)
    drop = [v for v in j.vars if v not in keep]
    return float(np.max(j.maximize(drop).values)) if drop else float(np.max(j.values))


def partition(factors):
    return float(np.sum(product_all(factors).values))


def _scores(graph, card):
    scores = {}
    for v in graph.nodes():
        nbrs = list(graph.neighbors(v))
        w = nx.Graph(graph.edges())
        w.add_edges_from(itertools.combinations(nbrs, 2))
        size = lambda c: float(np.prod([card[x] for x in c]))
        with_v = [c for c in nx.find_cliques(w) if v in c and all(u in c for u in nbrs)]
        w.remove_node(v)
        without = [c for c in nx.find_cliques(w) if all(u in c for u in nbrs)]
        mc = [size(c) for c in with_v]
        scores[v] = (size(without[0]), max(mc), sum(mc))
    return scores


def triangulate(edges, card, heuristic="H6"):
    """Edges of the triangulated graph (sorted pairs)."""
    g = nx.Graph(edges)
    if nx.is_chordal(g):
        return sorted(sorted(e) for e in g.edges())
    sc = _scores(g, card)
    f = {"H1": lambda s, v: s[0], "H2": lambda s, v: s[0] / card[v], "H3": lambda s, v: s[0] - s[1],
         "H4": lambda s, v: s[0] - s[2], "H5": lambda s, v: s[0] / s[1]}.get(heuristic, lambda s, v: s[0] / s[2])
    order = sorted(g.nodes(), key=lambda v: f(sc[v], v))
    h = nx.Graph(edges)
    out = nx.Graph(edges)
    for node in order:
        nb = list(h.neighbors(node))
        for a, b in itertools.combinations(nb, 2):
            h.add_edge(a, b)
            out.add_edge(a, b)
        h.remove_node(node)
    return sorted(sorted(e) for e in out.edges())


def jt_cliques(edges, card, heuristic="H6"):
    return sorted(sorted(c) for c in nx.find_cliques(nx.Graph(triangulate(edges, card, heuristic))))


def jt_edges(cliques):
    cl = [tuple(c) for c in cliques]
    if len(cl) < 2:
        return []
    g = nx.Graph()
    for a, b in itertools.combinations(cl, 2):
        g.add_edge(a, b, weight=-len(set(a) & set(b)))
    return list(nx.minimum_spanning_tree(g).edges())


def calibrate(factors, cliques, card, op="sum"):
    """Clique potentials (first clique covering each factor) calibrated by oracle.bp."""
    bags = [tuple(c) for c in cliques]
    pots = {}
    used = [False] * len(factors)
    for b in bags:
        f = OFactor(list(b), [card[v] for v in b], np.ones([card[v] for v in b]))
        for i, g in enumerate(factors):
            if not used[i] and set(g.vars) <= set(b):
                f = f.product(g)
                used[i] = True
        pots[b] = OFactor(list(b), [card[v] for v in b], f.aligned(list(b)))
    assert all(used), "a factor fits no clique"
    return OBP.calibrate(bags, jt_edges(bags), pots, op=op)
