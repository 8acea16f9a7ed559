"""numpy restatement of VariableElimination + predict (ORACLE — test infrastructure only).

  prune()            pgmpy/inference/base.py:154-212 (active trails: pgmpy/base/DAG.py:864-950,
                     ancestral graph DAG.py:1163-1186; pruned parents summed out + renormalised,
                     CPD.py:483-524)
  greedy_contract()  opt_einsum greedy strategy behind ExactInference.py:404-406
                     (private-index sums, then min size(out)-size(a)-size(b) pairs)
  eliminate()        classic VE loop ExactInference.py:141-244 in min-clique order
                     (EliminationOrder.py:146-157 cost on the working factors): munin C2 in ~0.1 s
  query()            ExactInference.py:246-440 (greedy path: drop all-evidence factors L383,
                     slice L352-365, contract, normalize L420, per-var marginals L430-433)
  map_query()        ExactInference.py:528-624 (joint, np.argmax first index, assignment)
  predict_rows() / predict_probability_rows()
                     DiscreteBayesianNetwork.py:731-989 per-row semantics
"""
import numpy as np

from .factor import OFactor


def active_trail_nodes(net, start, observed):
    observed = set(observed)
    anc = set(observed)
    stack = list(observed)
    while stack:
        n = stack.pop()
        for p in net.parents[n]:
            if p not in anc:
                anc.add(p)
                stack.append(p)
    visit = [(start, "up")]
    seen = set()
    active = set()
    while visit:
        node, d = visit.pop()
        if (node, d) in seen:
            continue
        seen.add((node, d))
        if node not in observed:
            active.add(node)
        if d == "up" and node not in observed:
            visit.extend((p, "up") for p in net.parents[node])
            visit.extend((c, "down") for c in net.children[node])
        elif d == "down":
            if node not in observed:
                visit.extend((c, "down") for c in net.children[node])
            if node in anc:
                visit.extend((p, "up") for p in net.parents[node])
    return active


def prune(net, variables, evidence_vars):
    """Kept nodes and their (possibly marginalised) factors."""
    dcon = set(evidence_vars)
    for v in variables:
        dcon |= active_trail_nodes(net, v, evidence_vars)
    targets = set(variables) | (set(evidence_vars) & dcon)
    keep = set(targets)
    stack = list(targets)
    while stack:
        n = stack.pop()
        for p in net.parents[n]:
            if p in dcon and p not in keep:
                keep.add(p)
                stack.append(p)
    factors = []
    for v in net.nodes:
        if v not in keep:
            continue
        f = net.factor(v)
        gone = [p for p in net.parents[v] if p not in keep]
        if gone:
            f = f.marginalize(gone)
            # TabularCPD.marginalize renormalises columns (CPD.py:449-481)
            s = f.values.sum(axis=0, keepdims=True)
            with np.errstate(invalid="ignore", divide="ignore"):
                f = OFactor(f.vars, f.card, f.values / s)
        factors.append(f)
    return keep, factors


def greedy_contract(operands, out_vars):
    """sum_{not out} prod operands via greedy pairwise np.einsum (small cases)."""
    ops = [(o.values, list(o.vars)) for o in operands]
    dims = {}
    for a, ls in ops:
        dims.update(zip(ls, a.shape))

    def needed(l, skip):
        return l in out_vars or any(l in ls for k, (_, ls) in enumerate(ops) if k not in skip)

    def esum(pairs, out):
        lab = {}
        for _, ls in pairs:
            for l in ls:
                lab.setdefault(l, len(lab))
        args = []
        for a, ls in pairs:
            args += [a, [lab[l] for l in ls]]
        return np.einsum(*args, [lab[l] for l in out])

    ops = [(esum([(a, ls)], [l for l in ls if needed(l, {k})]), [l for l in ls if needed(l, {k})])
           for k, (a, ls) in enumerate(ops)]
    while len(ops) > 1:
        best = None
        for i in range(len(ops)):
            for j in range(i + 1, len(ops)):
                li, lj = ops[i][1], ops[j][1]
                keep = [l for l in dict.fromkeys(li + lj) if needed(l, {i, j})]
                size = lambda ls: int(np.prod([dims[l] for l in ls])) if ls else 1
                key = (0 if set(li) & set(lj) else 1, size(keep) - size(li) - size(lj))
                if best is None or key < best[0]:
                    best = (key, i, j, keep)
        _, i, j, keep = best
        res = esum([ops[i], ops[j]], keep)
        ops = [o for k, o in enumerate(ops) if k not in (i, j)] + [(res, keep)]
    a, ls = ops[0]
    return esum([(a, ls)], list(out_vars))


def eliminate(operands, out_vars):
    """sum_{not out} prod operands by classic variable elimination, the loop of
    ExactInference.py:141-244 (_variable_elimination: for each variable in the order, the product of
    every working factor holding it, factor_product L200-215, then marginalize it out), with the order
    chosen as it goes: next the variable whose elimination clique (the union of the scopes of the
    working factors holding it) has the fewest states — EliminationOrder.py:146-157's MinWeight cost
    measured on the working factors.  For the big munin queries (C2: ~700 operands) where
    greedy_contract's all-pairs scan is too slow; the values equal it up to rounding."""
    import heapq
    import math

    dims = {}
    for o in operands:
        dims.update(zip(o.vars, o.card))
    work = {}   # factor id -> OFactor
    holders = {}  # variable -> set of factor ids
    for k, o in enumerate(operands):
        work[k] = o
        for v in o.vars:
            holders.setdefault(v, set()).add(k)
    nxt = len(operands)
    out = set(out_vars)

    def cost(v):
        scope = set()
        for k in holders[v]:
            scope.update(work[k].vars)
        return math.prod(dims[u] for u in scope)  # Python ints: no int64 overflow on wide scopes

    version = {v: 0 for v in holders}
    heap = [(cost(v), v, 0) for v in holders if v not in out]
    heapq.heapify(heap)
    while heap:
        c, v, ver = heapq.heappop(heap)
        if v not in holders or ver != version[v]:
            continue
        ks = sorted(holders.pop(v), key=lambda k: work[k].values.size)
        f = work.pop(ks[0])
        for k in ks[1:]:
            f = f.product(work.pop(k))
        f = f.marginalize([v])
        # every variable of the removed factors is in f's scope (their union minus v)
        for u in f.vars:
            holders[u].difference_update(ks)
            holders[u].add(nxt)
        work[nxt] = f
        nxt += 1
        for u in f.vars:
            if u not in out:
                version[u] += 1
                heapq.heappush(heap, (cost(u), u, version[u]))
    # what is left holds only output variables (or nothing: scalars)
    rest = sorted(work.values(), key=lambda o: o.values.size)
    f = rest[0]
    for g in rest[1:]:
        f = f.product(g)
    if not out_vars:
        return np.asarray(f.values.sum())
    return f.aligned(list(out_vars)) if set(f.vars) == set(out_vars) else \
        f.marginalize([u for u in f.vars if u not in out]).aligned(list(out_vars))


def joint(net, variables, evidence, contract=None):
    """Unnormalised joint over `variables` (in that order) given {var: state name}: the reference's
    contract result before normalize (ExactInference.py:349-420).  contract: greedy_contract (the
    reference's opt_einsum greedy strategy, default) or eliminate."""
    ev_no = {v: net.state_no(v, s) for v, s in evidence.items()}
    keep, factors = prune(net, variables, list(ev_no))
    ev_no = {v: s for v, s in ev_no.items() if v in keep}
    ops = []
    for f in factors:
        if all(v in ev_no for v in f.vars):
            continue
        ops.append(f.reduce({v: s for v, s in ev_no.items() if v in f.vars}))
    return (contract or greedy_contract)(ops, variables)


def query(net, variables, evidence, joint_out=True, contract=None):
    j = joint(net, variables, evidence, contract=contract)
    with np.errstate(invalid="ignore", divide="ignore"):
        j = j / j.sum()
    if joint_out:
        return j
    return {v: j.sum(axis=tuple(k for k in range(len(variables)) if k != i)) for i, v in enumerate(variables)}


def map_query(net, variables, evidence):
    j = joint(net, variables, evidence)
    with np.errstate(invalid="ignore", divide="ignore"):
        jn = j / j.sum()
    idx = int(np.argmax(jn))
    flat = np.sort(jn.ravel())[::-1]
    gap = float((flat[0] - flat[1]) / flat[0]) if flat.size > 1 and flat[0] > 0 else 1.0
    out = {}
    for i in reversed(range(len(variables))):
        c = j.shape[i]
        out[variables[i]] = net.states[variables[i]][idx % c]
        idx //= c
    return out, gap


def predict_probability_rows(net, missing, rows):
    """rows: list of {var: state name}. Returns [n_rows, sum card] marginals (missing order)."""
    out = []
    for ev in rows:
        m = query(net, missing, ev, joint_out=False)
        out.append(np.concatenate([m[v] for v in missing]))
    return np.array(out)


def predict_rows(net, missing, rows):
    return [map_query(net, missing, ev) for ev in rows]
