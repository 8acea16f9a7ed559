"""numpy restatement of junction-tree belief propagation (ORACLE — test infrastructure only).

Lauritzen-Spiegelhalter belief update as pgmpy/inference/ExactInference.py:770-805
(_update_beliefs: sigma = marginalize sender onto sepset; receiver *= sigma / mu
with 0/0 -> 0, DiscreteFactor.py:859-863; mu = sigma), scheduled as one
collect (leaves -> root) + one distribute (root -> leaves) sweep, the fixed point
_calibrate_junction_tree (L854-895) converges to.
"""
import numpy as np

from .factor import OFactor


def initial_potentials(net, bags):
    """Clique potentials: ones x product of CPDs assigned to the first bag covering their scope
    (the SURVEY.md §8(c) BP-oracle construction)."""
    assigned = {b: [] for b in bags}
    for v in sorted(net.nodes):
        scope = set([v] + list(net.parents[v]))
        for b in bags:
            if scope <= set(b):
                assigned[b].append(net.factor(v))
                break
    pots = {}
    for b in bags:
        f = OFactor(list(b), [net.card[v] for v in b], np.ones([net.card[v] for v in b]))
        for g in assigned[b]:
            f = f.product(g)
        pots[b] = OFactor(list(b), [net.card[v] for v in b], f.aligned(list(b)))
    return pots


def apply_evidence(net, pots, bags, evidence):
    """0/1 indicators of observed states into the first bag holding each variable."""
    pots = {b: p.copy() for b, p in pots.items()}
    for var, st in evidence.items():
        for b in bags:
            if var in b:
                ind = np.zeros(net.card[var])
                ind[net.state_no(var, st)] = 1.0
                p = pots[b].product(OFactor([var], [net.card[var]], ind))
                pots[b] = OFactor(list(b), pots[b].card, p.aligned(list(b)))
                break
    return pots


def calibrate(bags, edges, pots, op="sum"):
    beliefs = {b: pots[b].copy() for b in bags}
    adj = {b: [] for b in bags}
    for a, b in edges:
        adj[a].append(b)
        adj[b].append(a)
    root = bags[0]
    order, seen, queue = [], {root}, [root]
    while queue:
        p = queue.pop(0)
        for c in adj[p]:
            if c not in seen:
                seen.add(c)
                order.append((p, c))
                queue.append(c)
    seps = {}

    def send(src, dst):
        sep = [v for v in src if v in dst]
        drop = [v for v in src if v not in dst]
        sigma = beliefs[src].marginalize(drop) if op == "sum" else beliefs[src].maximize(drop)
        key = frozenset((src, dst))
        mu = seps.get(key)
        msg = sigma if mu is None else sigma.divide(mu)
        prod = beliefs[dst].product(msg)
        beliefs[dst] = OFactor(list(dst), beliefs[dst].card, prod.aligned(list(dst)))
        seps[key] = OFactor(sep, [beliefs[src].card[list(src).index(v)] for v in sep], sigma.aligned(sep))

    for p, c in reversed(order):
        send(c, p)
    for p, c in order:
        send(p, c)
    return beliefs, seps


def marginals(net, bags, beliefs):
    out = {}
    for var in sorted(net.nodes):
        for b in bags:
            if var in b:
                m = beliefs[b].marginalize([v for v in b if v != var]).values
                with np.errstate(invalid="ignore", divide="ignore"):
                    out[var] = m / m.sum()
                break
    return out


def check_batched_rows(net, bags, edges, beliefs_rows, ev_codes, ev_vars, rows, op="sum", rtol=1e-9):
    """Checker for a batched calibration: for each row r in `rows`, the row's findings (codes != 255 of
    `ev_codes[:, r]`) through apply_evidence + calibrate, compared entry by entry with the device's
    beliefs (`beliefs_rows[clique][i]` for rows[i], clique axes in the bag's order).  Returns
    (max relative error over entries > 1e-300, number of entries compared); raises AssertionError at
    the first clique outside `rtol`."""
    pots = initial_potentials(net, bags)
    worst, n = 0.0, 0
    for i, r in enumerate(rows):
        ev = {v: net.states[v][int(ev_codes[j, r])] for j, v in enumerate(ev_vars) if ev_codes[j, r] != 255}
        want, _ = calibrate(bags, edges, apply_evidence(net, pots, bags, ev), op=op)
        for b in bags:
            w = want[b].aligned(list(b)).ravel()
            g = beliefs_rows[tuple(b)][i]
            np.testing.assert_allclose(g, w, rtol=rtol, atol=1e-300,
                                       err_msg=f"row {r} clique {b[:4]}... evidence {ev}")
            nz = np.abs(w) > 1e-300
            if nz.any():
                worst = max(worst, float(np.max(np.abs(g[nz] - w[nz]) / np.abs(w[nz]))))
            n += w.size
    return worst, n
