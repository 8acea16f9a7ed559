"""Batched junction-tree calibration: one calibration per evidence row.

Each clique belief is a device tensor [clique vars..., ROW] with the evidence
row innermost (stride 1), so every message kernel is coalesced along rows
regardless of which clique axes it reduces.  Schedule = one collect
(leaves -> root) and one distribute (root -> leaves) sweep of
Lauritzen-Spiegelhalter belief update, the fixed point of the reference's
_calibrate_junction_tree (pgmpy/inference/ExactInference.py:770-895):

  collect   sigma = marg_{C_c \\ S}(beta_c);  beta_p *= sigma;            mu = sigma
  distribute sigma = marg_{C_p \\ S}(beta_p);  beta_c *= sigma / mu (0/0->0); mu = sigma

Findings enter as 0/1 indicators (pgm_indicator) multiplied into the first
clique that holds each observed variable.
Algorithmic bytes per calibration: 8 (4 sum|C| + 4 sum|S|).
"""
import numpy as np

from .. import engine as E


class BatchedCalibration:
    def __init__(self, bjt, beliefs, seps, n_rows):
        self.bjt = bjt
        self.beliefs = beliefs  # clique -> (tensor [labels..., ROW], labels)
        self.seps = seps
        self.n_rows = n_rows

    def clique_belief(self, clique, row):
        """Host copy of one row's belief, axes in the clique tuple's order (C-order flat)."""
        t, ls = self.beliefs[tuple(clique)]
        out = E.contract(t, ls + [E.ROW], None, None, [E.ROW] + list(clique), combine="copy")
        return E.to_host(out)[row].ravel()

    def marginal(self, var):
        """[n_rows, card] normalized marginal of `var` per row."""
        c = self.bjt.var_clique[var]
        t, ls = self.beliefs[c]
        m = E.contract(t, ls + [E.ROW], None, None, [E.ROW, var], reduce="sum", combine="copy")
        E.normalize_rows_(m, [E.ROW, var], E.ROW)
        return E.to_host(m)

    def marginals_device(self, variables=None):
        """{var: device [card, n_rows]} normalized marginals."""
        out = {}
        for var in (variables or self.bjt.variables):
            c = self.bjt.var_clique[var]
            t, ls = self.beliefs[c]
            m = E.contract(t, ls + [E.ROW], None, None, [var, E.ROW], reduce="sum", combine="copy")
            E.normalize_rows_(m, [var, E.ROW], E.ROW)
            out[var] = m
        return out


class BatchedJunctionTree:
    def __init__(self, jt):
        import networkx as nx

        self.jt = jt
        self.cliques = [tuple(c) for c in jt.nodes()]
        self.root = self.cliques[0]
        self.order = list(nx.bfs_edges(jt, self.root)) if len(self.cliques) > 1 else []
        self.pot = {}
        self.card = {}
        self.states = {}
        for c in self.cliques:
            f = jt.get_factors(c)
            self.pot[c] = (f._d(), list(f.variables))
            for v, k in zip(f.variables, f.cardinality):
                self.card[v] = int(k)
            self.states.update({v: list(s) for v, s in f.state_names.items()})
        self.var_clique = {}
        for c in self.cliques:
            for v in c:
                self.var_clique.setdefault(v, c)
        self.variables = sorted(self.var_clique, key=str)
        self.sizes = {c: int(np.prod([self.card[v] for v in c])) for c in self.cliques}

    def bytes_per_calibration(self):
        """SURVEY.md §8(d) C4 algorithmic bytes: 8 (4 sum|C| + 4 sum|S|)."""
        s = 0
        for p, c in self.order:
            s += int(np.prod([self.card[v] for v in c if v in p]))
        return 8 * (4 * sum(self.sizes.values()) + 4 * s)

    def calibrate_codes(self, codes, ev_vars, n_rows, operation="marginalize", err=None):
        """codes: device uint8 [len(ev_vars), n_rows] (255 = unobserved)."""
        red = "sum" if operation == "marginalize" else "max"
        R = E.ROW
        ones = E.to_device(np.ones(n_rows))
        beliefs = {}
        ev_by_clique = {}
        for j, v in enumerate(ev_vars):
            ev_by_clique.setdefault(self.var_clique[v], []).append((j, v))
        for c in self.cliques:
            t, ls = self.pot[c]
            b = E.contract(t, ls, ones, [R], ls + [R], combine="mul")
            for j, v in ev_by_clique.get(c, []):
                ind = E.indicator(codes[j], self.card[v], n_rows, err=err)
                E.contract(b, ls + [R], ind, [v, R], ls + [R], combine="mul", out=b)
            beliefs[c] = (b, ls)
        seps = {}
        for p, c in reversed(self.order):  # collect
            tc, lc = beliefs[c]
            tp, lp = beliefs[p]
            sep = [v for v in lc if v in p]
            sigma = E.contract(tc, lc + [R], None, None, sep + [R], reduce=red, combine="copy")
            E.contract(tp, lp + [R], sigma, sep + [R], lp + [R], combine="mul", out=tp)
            seps[(p, c)] = (sigma, sep)
        for p, c in self.order:  # distribute
            tc, lc = beliefs[c]
            tp, lp = beliefs[p]
            mu, sep = seps[(p, c)]
            sigma = E.contract(tp, lp + [R], None, None, sep + [R], reduce=red, combine="copy")
            ratio = E.contract(sigma, sep + [R], mu, sep + [R], sep + [R], combine="div")
            E.contract(tc, lc + [R], ratio, sep + [R], lc + [R], combine="mul", out=tc)
            seps[(p, c)] = (sigma, sep)
        return BatchedCalibration(self, beliefs, seps, n_rows)

    def encode(self, df):
        import pandas as pd

        ev_vars = list(df.columns)
        codes = np.empty((len(ev_vars), len(df)), dtype=np.uint8)
        for j, v in enumerate(ev_vars):
            st = self.states[v]
            col = df[v]
            isna = col.isna().to_numpy()
            c = np.asarray(pd.Categorical(col, categories=st).codes, dtype=np.int64)
            if ((c < 0) & ~isna).any():
                raise KeyError(f"unknown state for variable {v}")
            c[isna] = 255
            codes[j] = c
        return codes, ev_vars

    def calibrate_frame(self, df, operation="marginalize"):
        import torch

        from .batch import upload_codes

        codes, ev_vars = self.encode(df)
        d = upload_codes(codes)
        err = torch.zeros(1, dtype=torch.int32, device=d.device)
        cal = self.calibrate_codes(d, ev_vars, len(df), operation=operation, err=err)
        if int(err.item()) != 0:
            raise IndexError("evidence state code out of range")
        return cal
