"""Batched junction-tree calibration: one calibration per evidence row.

Each clique belief is a device tensor [clique vars..., ROW] with the evidence
row innermost (stride 1), so every message kernel is coalesced along rows
whatever clique axes it reduces.  The schedule is one collect (leaves -> root)
and one distribute (root -> leaves) sweep of Lauritzen-Spiegelhalter belief
update — the fixed point of the reference's _calibrate_junction_tree
(pgmpy/inference/ExactInference.py:770-895):

  collect    mu_c = marg_{C_c \\ S}(psi_c x findings_c x prod_{children k} mu_k)   (message to the parent;
             the clique-sized product is NOT written: the fused kernel's marginal-only mode)
  distribute sigma' = marg_{C_p \\ S}(beta_p);  beta_c = psi_c x findings_c x prod mu_k x sigma' / mu_c
             (0/0 -> 0, DiscreteFactor.py:859-863), written once

Findings enter as 0/1 indicators (pgm_indicator) of the first clique holding
each observed variable.  A compiled schedule (per batch size and evidence
columns) is a pgmpy_amd.program.Program: all buffers preallocated, replayed as
one HIP graph.  Algorithmic bytes per calibration: 8 (sum|C| + 4 sum|S|) — every belief written once,
every separator message and sigma' written and read once; SURVEY.md §8(d)'s 8 (4 sum|C| + 4 sum|S|)
counts the reference's schedule, which reads and writes each belief in both passes.
"""
import os

import numpy as np

from .. import _native as N
from .. import engine as E
from ..program import Program


class BatchedCalibration:
    def __init__(self, bjt, beliefs, seps, n_rows, marginals=None, done=None):
        self.bjt = bjt
        self.beliefs = beliefs  # clique -> (tensor [labels..., ROW], labels)
        self.seps = seps        # (parent, child) -> (tensor [sep..., ROW], sep labels)
        self.n_rows = n_rows
        self._marg = marginals or {}
        self._done = done  # calibrated on another stream (an in-flight lane): its completion event

    def wait(self):
        """Order the current stream after the calibration (a no-op unless it ran on an in-flight lane's
        stream); every accessor below calls it, a caller reading the tensors directly calls it first."""
        if self._done is not None:
            E._torch().cuda.current_stream().wait_event(self._done)
        return self

    def clique_belief(self, clique, row):
        """Host copy of one row's belief, axes in the clique tuple's order (C-order flat)."""
        self.wait()
        t, ls = self.beliefs[tuple(clique)]
        out = E.contract(t, ls + [E.ROW], None, None, [E.ROW] + list(clique), combine="copy")
        return E.to_host(out)[row].ravel()

    def clique_beliefs_rows(self, rows):
        """{clique: [len(rows), Π card]} host copies of the given rows' beliefs, axes in each clique
        tuple's order (C-order flat) — one device pass and one download per clique."""
        self.wait()
        torch = E._torch()
        idx = torch.as_tensor(np.asarray(rows, dtype=np.int64), device=E.device())
        out = {}
        for c, (t, ls) in self.beliefs.items():
            full = E.contract(t, ls + [E.ROW], None, None, list(c) + [E.ROW], combine="copy")
            sel = full.reshape(-1, self.n_rows).index_select(1, idx)
            out[c] = E.to_host(sel).T.copy()
        return out

    def marginal(self, var):
        """[n_rows, card] normalized marginal of `var` per row."""
        self.wait()
        if var in self._marg:
            return E.to_host(self._marg[var]).T.copy()
        c = self.bjt.var_clique[var]
        t, ls = self.beliefs[c]
        m = E.contract(t, ls + [E.ROW], None, None, [E.ROW, var], reduce="sum", combine="copy")
        E.normalize_rows_(m, [E.ROW, var], E.ROW)
        return E.to_host(m)

    def marginals_device(self):
        self.wait()
        return dict(self._marg)


# a clique's finalising pass stores its child's update ratio sigma'/mu instead of sigma' where it can
# (BPSchedule.premarginal); A/B knob PGM_BP_RATIO=0
RATIO_PREMARG = os.environ.get("PGM_BP_RATIO", "1") != "0"


class _SepFromRatio:
    """A sepset belief sigma' the schedule did not store: the child's update ratio r = sigma'/mu and its
    message mu; sigma' = r x mu (exact where mu = 0: the parent's belief then holds the factor mu, so
    sigma' = 0 = r x mu), made on first use (outside the compiled program)."""

    def __init__(self, ratio, mu, sl):
        self.ratio, self.mu, self.sl = ratio, mu, sl
        self._t = None

    def __getitem__(self, i):
        if self._t is None:
            self._t = E.product_n([(self.ratio, self.sl), (self.mu, self.sl)], self.sl)
        return (self._t, self.sl[:-1])[i]

    def __iter__(self):
        return iter((self[0], self[1]))


def _aggregate(prog, small, clique_labels, scope_size):
    """Multiply the findings / messages entering a clique bottom-up over their scopes.

    Operands with the same scope are multiplied at that scope; each scope's product is folded
    into the smallest containing scope among the operands' scopes (still separator-sized), so the
    clique-sized product reads only the maximal scopes' aggregates (pathfinder's root: 57 child
    messages, 46 of them over one variable -> 3 operands).  Returns [(tensor, labels)]."""
    R = E.ROW
    groups = {}
    for t, labels in small:
        sc = tuple(v for v in clique_labels if v in labels)
        groups.setdefault(sc, []).append((t, list(labels)))
    order = sorted(groups, key=lambda sc: (scope_size(sc), len(sc)))
    folded = {sc: [] for sc in order}
    top = []
    for i, sc in enumerate(order):
        items = groups[sc] + folded[sc]
        bigger = [t for t in order[i + 1:] if set(sc) < set(t)]
        if len(items) == 1:
            agg = items[0]
        else:
            agg = (prog.product_n(items, list(sc) + [R]), list(sc) + [R])
        if bigger:
            folded[min(bigger, key=lambda t: (scope_size(t), len(t)))].append(agg)
        else:
            top.append(agg)
    return top


class BPSchedule:
    """A compiled batched calibration for fixed (n_rows, evidence columns, operation)."""

    def __init__(self, bjt, n_rows, ev_vars, operation="marginalize", marginals=True, graph=True, levels=True):
        import torch

        self.bjt = bjt
        self.n_rows = n_rows
        self.ev_vars = list(ev_vars)
        red = "sum" if operation == "marginalize" else "max"
        R = E.ROW
        # levelled: independent cliques' small products / separator marginals share one launch per
        # dependency level (collect: tree height; distribute: depth; r01: 408 -> 170 launches)
        prog = Program(levels=levels)
        dev = E.device()
        self.codes = torch.empty((max(1, len(self.ev_vars)), n_rows), dtype=torch.uint8, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        ev_by_clique = {}
        for j, v in enumerate(self.ev_vars):
            ev_by_clique.setdefault(bjt.var_clique[v], []).append((j, v))
        children = {c: [] for c in bjt.cliques}
        parent = {}
        for p, c in bjt.order:
            children[p].append(c)
            parent[c] = p
        beliefs, msgs, seps = {}, {}, {}
        size = {v: bjt.card[v] for v in bjt.card}

        def scope_size(sc):
            return int(np.prod([size[v] for v in sc])) if sc else 1

        kids = {}
        for p, c in bjt.order:
            kids.setdefault(p, []).append(c)

        def largest_kid_scope(c):
            """The largest separator scope (in c's variable order) of c's children: the marginal of
            c's final belief the distribute sweep needs first."""
            lc = bjt.pot[c][1]
            scs = {tuple(v for v in lc if v in k) for k in kids[c]}
            return max(scs, key=lambda x: (scope_size(x), len(x)))

        def premarginal(c, ops, labels, out=None, kinds=None):
            """c's finalising pass: its belief (into `out`) with the marginal onto its largest child scope S.
            When exactly one child k has scope S, k's message mu_k is one of the pass's operands and no other
            child scope needs sigma'(S) to be derived from, the pass stores k's update ratio sigma'(S) / mu_k
            instead (PGM_PRODN_MDIV, 0/0 -> 0): k's own pass then reads one separator-sized operand instead of
            sigma' and mu_k (r05).  Returns (belief, (S, marginal, k or None))."""
            sc = largest_kid_scope(c)
            base = list(kinds) if kinds is not None else [N.PRODN_MUL] * len(ops)
            ks = [k for k in kids[c] if set(msgs[k][1][:-1]) == set(sc)]
            idx = None
            if RATIO_PREMARG and len(ks) == 1:
                idx = next((i for i, (t_, _) in enumerate(ops) if t_ is msgs[ks[0]][0] and base[i] == N.PRODN_MUL), None)
                other = {frozenset(msgs[q][1][:-1]) for q in kids[c]} - {frozenset(sc)}
                for s_ in other:  # every other child scope inside S still finds a sigma' to come from
                    if s_ <= set(sc) and not any(s_ < t_ for t_ in other):
                        idx = None
                if idx is not None:
                    if out is None:
                        out = E.empty([bjt.card[v] for v in labels] + [n_rows])
                    mk = list(base)
                    mk[idx] = N.PRODN_MDIV
                    ok = E.prepare_product_n_marginal(ops, labels + [R], list(sc) + [R], out, mk)[5]
                    if ok:
                        bt, m, _ = prog.product_n_marginal(ops, labels + [R], list(sc) + [R], out=out, kinds=mk,
                                                           reduce=red)
                        return bt, (sc, m, ks[0])
            bt, m, _ = prog.product_n_marginal(ops, labels + [R], list(sc) + [R], out=out, kinds=kinds, reduce=red)
            return bt, (sc, m, None)

        premarg = {}  # clique -> (scope, marginal of its final belief or a child's update ratio, that child)
        operands = {}  # clique -> its collect operands: [psi_c] + aggregated findings / child messages
        # collect: post-order (children before parents).  A clique's message to its parent is the
        # marginal of psi_c x aggregates computed WITHOUT writing the clique-sized product (the
        # fused kernel's marginal-only mode): the belief is written once, in distribute.  The root's
        # belief is final after collect (its largest child-separator marginal in the same pass).
        post = [c for _, c in reversed(bjt.order)] + [bjt.root]
        for c in post:
            t, ls = bjt.pot[c]
            small = []  # (tensor, labels incl. R): findings and child messages, all over subsets of c
            for j, v in ev_by_clique.get(c, []):
                small.append((prog.indicator(self.codes[j], bjt.card[v], n_rows, err=self.err), [v, R]))
            for k in children[c]:
                small.append(msgs[k])
            # the clique's passes read its findings and child messages directly when one fused pass takes
            # them all (and, below the root, sigma' / mu as well in distribute): no pre-multiplied
            # aggregate is written and read again (r05: 530 MB written + 743 MB read per 4,000-row
            # sweep of pathfinder went to aggregates); more operands than that are multiplied bottom-up
            # over their scopes first (_aggregate)
            direct = 1 + len(small) + (2 if c in parent else 0) <= N.PM_MAX_OPS
            ops = [(t, ls)] + (list(small) if direct else _aggregate(prog, small, ls, scope_size))
            if len(ops) == 1:
                ops.append((E.to_device(np.ones(n_rows)), [R]))  # broadcast psi over the rows
            operands[c] = ops
            if c in parent:
                sep = [v for v in ls if v in parent[c]]
                # the message from the findings / child messages themselves when the fused pass takes
                # them all: the aggregates (distribute's operands) are then off collect's critical path
                # (one dependency level less per clique whose inputs share a scope; +1-2 %, r03ad)
                mops = ops
                if len(ops) - 1 < len(small) and 1 + len(small) <= N.PM_MAX_OPS:
                    mops = [(t, ls)] + list(small)
                bt, m, _ = prog.product_n_marginal(mops, ls + [R], sep + [R], reduce=red, store=False)
                beliefs[c] = (bt, ls)  # the buffer distribute writes (the fallback path filled it already)
                msgs[c] = (m, sep + [R])
            elif c in kids:
                bt, premarg[c] = premarginal(c, ops, ls)
                beliefs[c] = (bt, ls)
            else:
                beliefs[c] = (prog.product_n(ops, ls + [R]), ls)
        # distribute: root -> leaves; one sigma' per distinct separator scope of a parent, each
        # marginalised from the smallest already-computed containing scope (or the belief).  A child's
        # final belief beta_c = psi_c x aggregates x sigma'/mu (0/0 -> 0) is written in ONE pass from
        # its collect operands (the separator-sized ratio folded into them), with its own largest
        # child-scope marginal in the same pass — the reference's beta_c *= sigma'/mu
        # (ExactInference.py:798-802) on a belief that was never materialised before.
        final = {bjt.root: (operands[bjt.root], None)}  # clique -> (operands, kinds) its belief is the product of

        def finalise(p, c, sigma=None, ratio=None):
            """c's final belief psi_c x operands x sigma'/mu_c in one pass (with its own premarginal when it
            has children); `ratio` = sigma'/mu_c already made by the parent's pass."""
            tc, lc = beliefs[c]
            mu, sl = msgs[c]
            if ratio is not None and len(operands[c]) + 1 <= N.PM_MAX_OPS:
                ops_c = operands[c] + [(ratio, sl)]
                kinds = None
            elif ratio is not None:  # folded into the aggregates
                ops_c = [operands[c][0]] + _aggregate(prog, operands[c][1:] + [(ratio, sl)], lc, scope_size)
                kinds = None
            elif len(operands[c]) + 2 <= N.PM_MAX_OPS:  # sigma' / mu as a ratio operand pair (0/0 -> 0)
                ops_c = operands[c] + [(sigma, sl), (mu, sl)]
                kinds = [N.PRODN_MUL] * len(operands[c]) + [N.PRODN_RATIO, N.PRODN_DEN]
            else:  # the separator-sized ratio folded into the aggregates
                r_ = prog.product_n([(sigma, sl), (mu, sl)], sl, kinds=[N.PRODN_RATIO, N.PRODN_DEN])
                ops_c = [operands[c][0]] + _aggregate(prog, operands[c][1:] + [(r_, sl)], lc, scope_size)
                kinds = None
            final[c] = (ops_c, kinds)
            if c in kids:
                _, premarg[c] = premarginal(c, ops_c, lc, out=tc, kinds=kinds)
            else:
                prog.product_n(ops_c, lc + [R], out=tc, kinds=kinds)
            seps[(p, c)] = (sigma, sl[:-1]) if ratio is None else _SepFromRatio(ratio, mu, sl)
        for p in [bjt.root] + [c for _, c in bjt.order]:
            if p not in kids:
                continue
            tp, lp = beliefs[p]
            scopes = {}
            for c in kids[p]:
                scopes.setdefault(tuple(msgs[c][1][:-1]), []).append(c)
            have = {tuple(lp): tp}
            ratio_kid = None
            if p in premarg:
                sc0, m0, ratio_kid = premarg[p]
                if ratio_kid is None:
                    have[tuple(sc0)] = m0
            ordered = sorted(scopes, key=lambda x: -scope_size(x))
            for si, sc in enumerate(ordered):
                if ratio_kid is not None and scopes[sc] == [ratio_kid]:
                    finalise(p, ratio_kid, ratio=premarg[p][1])
                    continue
                if sc in have:
                    sigma = have[sc]
                else:
                    src = min((h for h in have if set(sc) <= set(h)), key=scope_size)
                    sigma = None
                    if src == tuple(lp):  # not from the belief (a clique-sized read): from its operands,
                        fops, fk = final[p]  # marginal only (the fused kernel writes nothing but sigma')
                        # a second scope that would also come from the operands: both in one pass
                        partner = next((s2 for s2 in ordered[si + 1:] if s2 not in have and not set(s2) <= set(sc)
                                        and all(not set(s2) <= set(h) for h in have if h != tuple(lp))), None)
                        two = None
                        if partner is not None:
                            two = prog.product_n_marginals(fops, lp + [R], list(sc) + [R], list(partner) + [R],
                                                           out=tp, kinds=fk, reduce=red)
                        if two is not None:
                            sigma, have[partner] = two
                        else:
                            d_, p_, o_, ms_, M_, ok = E.prepare_product_n_marginal(fops, lp + [R], list(sc) + [R],
                                                                                   tp, fk, store=False)
                            if ok:
                                _, sigma, _ = prog.product_n_marginal(fops, lp + [R], list(sc) + [R], out=tp,
                                                                      kinds=fk, reduce=red, store=False)
                    if sigma is None and src != tuple(lp):
                        # a second scope whose smallest computed container is the same source: both marginals
                        # in one read of it (C4's root child scopes, 129 / 64 MB sources read once, not twice:
                        # 3.45 -> 3.40 MB per calibration, +1 % at 4,000 rows; profiles/r05ai/)
                        partner = next((s2 for s2 in ordered[si + 1:] if s2 not in have
                                        and not set(s2) <= set(sc) and not set(sc) <= set(s2)
                                        and min((h for h in have if set(s2) <= set(h)), key=scope_size) == src), None)
                        if partner is not None:
                            two = prog.product_n_marginals([(have[src], list(src) + [R])], list(src) + [R],
                                                           list(sc) + [R], list(partner) + [R], out=have[src],
                                                           reduce=red)
                            if two is not None:
                                sigma, have[partner] = two
                    if sigma is None:
                        sigma = prog.contract(have[src], list(src) + [R], None, None, list(sc) + [R], reduce=red,
                                              combine="copy")
                    have[sc] = sigma
                for c in scopes[sc]:
                    finalise(p, c, sigma=sigma)
        marg = {}
        if marginals:
            for var in bjt.variables:
                t, ls = beliefs[bjt.var_clique[var]]
                m = prog.contract(t, ls + [R], None, None, [var, R], reduce="sum", combine="copy")
                z = prog.contract(m, [var, R], None, None, [R], reduce="sum", combine="copy")
                prog.contract(m, [var, R], z, [R], [var, R], combine="div_raw", out=m)
                marg[var] = m
        self.prog = prog
        self.beliefs = beliefs
        self.seps = seps
        self.marg = marg
        if graph:
            prog.capture()

    def run(self, codes=None):
        """codes: device uint8 [len(ev_vars), n_rows] (copied into the schedule's input buffer)."""
        from .. import _native as N

        L = N.lib()
        s = N.stream_handle()
        N.check(L.pgm_memset(N.ptr(self.err), 0, 4, s), "memset")
        if codes is not None and len(self.ev_vars):
            if tuple(codes.shape) != tuple(self.codes.shape) or not codes.is_contiguous():
                raise ValueError(f"codes must be a contiguous uint8 [{len(self.ev_vars)}, {self.n_rows}] tensor")
            N.check(L.pgm_memcpy_d2d(N.ptr(self.codes), N.ptr(codes), codes.numel(), s), "memcpy_d2d")
        self.prog.run()
        return BatchedCalibration(self.bjt, self.beliefs, self.seps, self.n_rows, self.marg)


class BatchedJunctionTree:
    """inflight (r05): calibrate_codes keeps this many calibration batches in flight — k compiled schedules
    (own buffers) taken round robin, each on its own stream ordered after the caller's, so one batch's
    first levels overlap the previous batch's last (C4, 2 in flight: 1.16 -> 1.31 M calibrations/s at
    1,000 rows, 1.31 -> 1.41 M at 4,000; profiles/r05y/).  A returned calibration stays valid for the
    next k - 1 calls; its accessors order the caller's stream after it."""

    def __init__(self, jt, inflight=1):
        import networkx as nx

        self.jt = jt
        self.cliques = [tuple(c) for c in jt.nodes()]
        self.root = self.cliques[0]
        self.order = list(nx.bfs_edges(jt, self.root)) if len(self.cliques) > 1 else []
        self.pot = {}
        self.card = {}
        self.states = {}
        # (r03 also tried a clique layout with the variables most separators share first: slower overall,
        # profiles/r03m_*, r03n_*)
        for c in self.cliques:
            f = jt.get_factors(c)
            labels = list(f.variables)
            self.pot[c] = (f._d(), labels)
            for v, k in zip(f.variables, f.cardinality):
                self.card[v] = int(k)
            self.states.update({v: list(s) for v, s in f.state_names.items()})
        self.var_clique = {}
        for c in self.cliques:
            for v in c:
                self.var_clique.setdefault(v, c)
        self.variables = sorted(self.var_clique, key=str)
        self.sizes = {c: int(np.prod([self.card[v] for v in c])) for c in self.cliques}
        self._schedules = {}
        self.inflight = max(1, int(inflight))
        self._lane = 0
        self._lane_streams = {}

    def _sum_sep(self):
        return sum(int(np.prod([self.card[v] for v in c if v in p])) for p, c in self.order)

    def bytes_per_calibration(self):
        """Algorithmic HBM bytes of this schedule per calibration: 8 (sum|C| + 4 sum|S|) (each belief
        written once in distribute; each separator message and sigma' written and read once)."""
        return 8 * (sum(self.sizes.values()) + 4 * self._sum_sep())

    def reference_bytes_per_calibration(self):
        """SURVEY.md §8(d) C4's figure for the two-pass schedule that reads and writes every belief
        in both sweeps: 8 (4 sum|C| + 4 sum|S|)."""
        return 8 * (4 * sum(self.sizes.values()) + 4 * self._sum_sep())

    def schedule(self, n_rows, ev_vars, operation="marginalize", marginals=True, graph=True, lane=0):
        key = (n_rows, tuple(ev_vars), operation, marginals, graph, lane)
        sch = self._schedules.get(key)
        if sch is None:
            sch = BPSchedule(self, n_rows, ev_vars, operation, marginals, graph)
            self._schedules[key] = sch
        return sch

    def calibrate_codes(self, codes, ev_vars, n_rows, operation="marginalize", err=None, marginals=False):
        """codes: device uint8 [len(ev_vars), n_rows] (255 = unobserved)."""
        if self.inflight == 1:
            sch = self.schedule(n_rows, ev_vars, operation, marginals)
            cal = sch.run(codes)
            if err is not None:
                err.copy_(sch.err)
            return cal
        torch = E._torch()
        lane = self._lane
        self._lane = (lane + 1) % self.inflight
        sch = self.schedule(n_rows, ev_vars, operation, marginals, lane=lane)
        caller = torch.cuda.current_stream()
        st = self._lane_streams.get(lane)
        if st is None:
            st = self._lane_streams[lane] = torch.cuda.Stream()
        # after what the caller queued: the codes' producer, and its reads of this lane's previous results
        st.wait_stream(caller)
        if hasattr(codes, "record_stream"):  # the caller may drop its codes tensor before the lane reads it
            codes.record_stream(st)
        with torch.cuda.stream(st):
            cal = sch.run(codes)
            if err is not None:
                err.copy_(sch.err)
            done = torch.cuda.Event()
            done.record(st)
        cal._done = done
        if err is not None:
            caller.wait_event(done)
        return cal

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
        """One calibration per row of df (state names; NaN = unobserved).  encode() has already
        rejected unknown states, so the codes are in range; one at a time (inflight 1) the device's
        range flag is read back as well, k in flight skips that synchronisation (it would serialise
        the lanes)."""
        from .batch import download, upload_codes

        codes, ev_vars = self.encode(df)
        d = upload_codes(codes)
        if self.inflight > 1:
            return self.calibrate_codes(d, ev_vars, len(df), operation, marginals=True)
        sch = self.schedule(len(df), ev_vars, operation)
        cal = sch.run(d)
        if int(download(sch.err)[0]) != 0:
            raise IndexError("evidence state code out of range")
        return cal
