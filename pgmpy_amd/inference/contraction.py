"""Greedy pairwise sum-product contraction (replaces opt_einsum.contract(..., optimize="greedy")).

Reference call sites: pgmpy/inference/ExactInference.py:404-406 (the default
VariableElimination.query path) and pgmpy/factors/base.py:106
(factor_sum_product).  opt_einsum (pyproject.toml:36, ">=3.3", unpinned, not
vendored) plans a greedy path; its published greedy strategy is restated here:

  1. sum every label that occurs in exactly one operand and not in the output;
  2. repeatedly contract the pair of operands that share a label and minimise
     size(result) - size(a) - size(b), keeping a label in the result while any
     other operand or the output still needs it;
  3. with no pair sharing a label left, take outer products of the two
     smallest operands.

The executed path is the cheaper (by an MI355X cost estimate) of that greedy path and a
min-weight variable-elimination path (elimination_path; on munin's C2 query 32 MB / 18 MFLOP
instead of greedy's 1.5 GB / 19.9 GFLOP) — the values do not depend on the path beyond rounding.

Every pairwise step is ONE fused product+marginalize kernel (pgm_contract,
combine=MUL, reduce=SUM): the broadcast product is never materialised.  Steps
that are dense GEMMs (shared summed variables of total cardinality >= 8, each
side keeping >= 16 states) run on FP64 MFMA instead (pgm_gemm, engine.pair_gemm).  A
``ROW`` label (evidence rows) is just another kept label, so the same planner
and executor run single queries (C2) and row batches.
"""
import heapq
import os
import threading
from collections import OrderedDict
from functools import partial
from itertools import count

import numpy as np

from .. import engine as E


def _size(labels, dims):
    s = 1
    for l in labels:
        s *= int(dims[l])
    return s


def greedy_path(operand_labels, out_labels, dims):
    """Plan the contraction.

    Returns (steps, final_id): steps are ("reduce", i, keep, new_id) or
    ("pair", i, j, keep, new_id) over operand ids (inputs are 0..n-1)."""
    out_set = set(out_labels)
    ops = {i: list(dict.fromkeys(ls)) for i, ls in enumerate(operand_labels)}
    holders = {}
    for i, ls in ops.items():
        for l in ls:
            holders.setdefault(l, set()).add(i)
    steps = []
    ids = count(len(operand_labels))

    def kept(labels, exclude):
        return [l for l in labels if l in out_set or len(holders[l] - exclude) > 0]

    # 1. private labels
    for i in list(ops):
        ls = ops[i]
        keep = kept(ls, {i})
        if keep != ls:
            nid = next(ids)
            steps.append(("reduce", i, keep, nid))
            for l in ls:
                holders[l].discard(i)
            for l in keep:
                holders[l].add(nid)
            del ops[i]
            ops[nid] = keep

    def pair_entry(i, j):
        li, lj = ops[i], ops[j]
        union = list(dict.fromkeys(li + lj))
        keep = kept(union, {i, j})
        cost = _size(keep, dims) - _size(li, dims) - _size(lj, dims)
        return (cost, min(i, j), max(i, j), keep)

    heap = []
    seen = set()

    def push_pairs(i):
        partners = set()
        for l in ops[i]:
            partners |= holders[l]
        partners.discard(i)
        for j in partners:
            key = (min(i, j), max(i, j))
            if key in seen:
                continue
            seen.add(key)
            c, a, b, keep = pair_entry(i, j)
            heapq.heappush(heap, (c, a, b, keep))

    for i in list(ops):
        push_pairs(i)
    while len(ops) > 1:
        entry = None
        while heap:
            c, a, b, keep = heapq.heappop(heap)
            if a in ops and b in ops:
                entry = (a, b, keep)
                break
        if entry is None:
            # disconnected operands: outer product of the two smallest
            sizes = sorted(ops, key=lambda k: (_size(ops[k], dims), k))
            a, b = sizes[0], sizes[1]
            union = list(dict.fromkeys(ops[a] + ops[b]))
            entry = (a, b, kept(union, {a, b}))
        a, b, keep = entry
        nid = next(ids)
        steps.append(("pair", a, b, keep, nid))
        for l in ops[a] + ops[b]:
            holders[l].discard(a)
            holders[l].discard(b)
        for l in keep:
            holders[l].add(nid)
        del ops[a], ops[b]
        ops[nid] = keep
        push_pairs(nid)
    (final_id,) = ops.keys() if ops else (None,)
    return steps, final_id


def elimination_path(operand_labels, out_labels, dims, depth_aware=False):
    """A contraction path from a variable-elimination order (returns greedy_path's format).

    opt_einsum's greedy rule (greedy_path) looks one pairwise step ahead; on munin's C2 query it
    builds 36 M-entry intermediates and does 19.9 GFLOP.  Classic VE instead eliminates, at each
    step, the variable whose elimination clique is smallest — the MinWeight heuristic
    (pgmpy/inference/EliminationOrder.py:136-150: the product of the cardinalities of the
    variable's neighbours) measured on the current factors — multiplying the factors that hold it
    smallest-first and summing it out with the last product.  On C2 that is 18 MFLOP and 32 MB
    with a 168 K-entry largest intermediate.  Values do not depend on the path beyond rounding.
    depth_aware: the factors holding the variable are multiplied shallowest-first (then smallest) —
    a balanced product tree instead of a chain, so fewer dependency levels (one launch each in a
    compiled program) for somewhat larger intermediates (C2: 23 levels / 49 MB against 29 / 32 MB)."""
    out_set = set(out_labels)
    ops = {i: list(dict.fromkeys(ls)) for i, ls in enumerate(operand_labels)}
    dep = {i: 0 for i in ops}
    holders = {}
    for i, ls in ops.items():
        for l in ls:
            holders.setdefault(l, set()).add(i)
    steps = []
    ids = count(len(operand_labels))

    def kept(labels, exclude):
        return [l for l in labels if l in out_set or len(holders[l] - exclude) > 0]

    def retire(olds, keep, kind, extra=()):
        nid = next(ids)
        steps.append((kind,) + tuple(olds[:1] if kind == "reduce" else olds) + (keep, nid))
        touched = set()
        dep[nid] = 1 + max(dep[o] for o in olds)
        for o in olds:
            for l in ops[o]:
                holders[l].discard(o)
                touched.add(l)
            del ops[o]
        for l in keep:
            holders[l].add(nid)
        ops[nid] = keep
        return nid, touched

    def order_key(i):
        return (dep[i], _size(ops[i], dims), i) if depth_aware else (_size(ops[i], dims), i)

    for i in list(ops):  # 1. private labels, as in greedy_path
        keep = kept(ops[i], {i})
        if keep != ops[i]:
            retire([i], keep, "reduce")

    def weight(v):
        nb = set()
        for i in holders[v]:
            nb.update(ops[i])
        return _size(nb, dims)

    heap, ver, done = [], {}, set()
    for v, h in holders.items():
        if v not in out_set and h:
            ver[v] = 0
            heapq.heappush(heap, (weight(v), 0, str(v), v))
    while heap:  # 2. eliminate the minimum-weight variable (lazy re-weighing)
        w, vv, _, v = heapq.heappop(heap)
        if v in done or ver.get(v) != vv or not holders[v]:
            continue
        cw = weight(v)
        if cw != w:
            ver[v] += 1
            heapq.heappush(heap, (cw, ver[v], str(v), v))
            continue
        done.add(v)
        inv = sorted(holders[v], key=order_key)
        touched = set()
        while len(inv) > 1:
            a, b = inv[0], inv[1]
            nid, t = retire([a, b], kept(list(dict.fromkeys(ops[a] + ops[b])), {a, b}), "pair")
            touched |= t
            inv = sorted([nid] + inv[2:], key=order_key)
        if v in ops[inv[0]]:
            _, t = retire([inv[0]], [l for l in ops[inv[0]] if l != v], "reduce")
            touched |= t
        for l in touched:
            if l not in done and l not in out_set and holders[l]:
                ver[l] = ver.get(l, 0) + 1
                heapq.heappush(heap, (weight(l), ver[l], str(l), l))
    while len(ops) > 1:  # 3. what is left shares only output labels: smallest first
        a, b = sorted(ops, key=order_key)[:2]
        retire([a, b], kept(list(dict.fromkeys(ops[a] + ops[b])), {a, b}), "pair")
    (final_id,) = ops.keys() if ops else (None,)
    return steps, final_id


def order_path(operand_labels, out_labels, dims, order):
    """A contraction path that eliminates variables in a GIVEN order (classic variable elimination,
    pgmpy/inference/ExactInference.py:141-244, whose order comes from an EliminationOrder heuristic or
    the caller): for each variable, the live operands holding it are multiplied smallest-first and
    the variable is summed (or maxed) out with the last product; a label no other operand or the
    output needs is summed in the same pass.  Labels the order omits are eliminated afterwards,
    then what is left (output labels only) is multiplied smallest-first.  greedy_path's format."""
    out_set = set(out_labels)
    ops = {i: list(dict.fromkeys(ls)) for i, ls in enumerate(operand_labels)}
    holders = {}
    for i, ls in ops.items():
        for l in ls:
            holders.setdefault(l, set()).add(i)
    steps = []
    ids = count(len(operand_labels))

    def kept(labels, exclude):
        return [l for l in labels if l in out_set or len(holders[l] - exclude) > 0]

    def retire(olds, keep, kind):
        nid = next(ids)
        steps.append((kind,) + tuple(olds) + (keep, nid))
        for o in olds:
            for l in ops[o]:
                holders[l].discard(o)
            del ops[o]
        for l in keep:
            holders[l].add(nid)
        ops[nid] = keep
        return nid

    def size_key(i):
        return (_size(ops[i], dims), i)

    rest = [l for l in holders if l not in out_set and l not in set(order)]
    for v in list(order) + rest:
        if v in out_set or not holders.get(v):
            continue
        inv = sorted(holders[v], key=size_key)
        while len(inv) > 1:
            a, b = inv[0], inv[1]
            nid = retire([a, b], kept(list(dict.fromkeys(ops[a] + ops[b])), {a, b}), "pair")
            inv = sorted([nid] + inv[2:], key=size_key)
        if v in ops[inv[0]]:
            retire([inv[0]], [l for l in ops[inv[0]] if l != v], "reduce")
    while len(ops) > 1:
        a, b = sorted(ops, key=size_key)[:2]
        retire([a, b], kept(list(dict.fromkeys(ops[a] + ops[b])), {a, b}), "pair")
    (final_id,) = ops.keys() if ops else (None,)
    return steps, final_id


def path_cost(steps, operand_labels, dims):
    """(bytes, flops, depth) of a path: 8 (|A| + |B| + |C|) bytes and 2 |index space| flops per
    pairwise step, |A| + |C| per reduction; depth = the longest chain of dependent steps."""
    labels = {i: list(dict.fromkeys(ls)) for i, ls in enumerate(operand_labels)}
    depth = {i: 0 for i in labels}
    nbytes = flops = maxd = 0
    for st in steps:
        ins, keep, nid = st[1:-2], st[-2], st[-1]
        nbytes += 8 * (sum(_size(labels[i], dims) for i in ins) + _size(keep, dims))
        space = list(dict.fromkeys(l for i in ins for l in labels[i]))
        flops += (1 if st[0] == "reduce" else 2 if st[0] == "pair" else len(ins)) * _size(space, dims)
        d = max(depth[i] for i in ins) + 1
        labels[nid], depth[nid] = keep, d
        maxd = max(maxd, d)
    return nbytes, flops, maxd


def choose_path(operand_labels, out_labels, dims):
    """The cheapest of opt_einsum's greedy path and the min-weight elimination path (product chains,
    or shallowest-first product trees), by an MI355X estimate: bytes at 3 TB/s + flops at 15 TFLOP/s
    + 5 us per dependency level (one batched launch per level in a compiled program: ~5 us launch to
    launch for these small steps, profiles/r03g_c2_levels.txt)."""
    best = None
    for planner in (greedy_path, elimination_path, partial(elimination_path, depth_aware=True)):
        steps, final_id = planner(operand_labels, out_labels, dims)
        nbytes, flops, depth = path_cost(steps, operand_labels, dims)
        est = nbytes / 3e12 + flops / 15e12 + depth * 5e-6
        if best is None or est < best[0]:
            best = (est, steps, final_id)
    return best[1], best[2]


# r06: the pairwise steps of a compiled single-row path fused into n-ary steps (fuse_path) of at most
# FUSE_BUDGET index-space entries each: fewer dependency levels, i.e. fewer dependent launches per query
# (512 Ki / 512 since the n-ary kernels' lanes stride over the outer reduction dims only and walk the inner
# ones as literal loops: C2 16 -> 11 launches, 85-86.5 -> 78.8 us per query; 1 Mi entries: slower again,
# profiles/r06ab/, r06ad/.  64 Ki / 64 before: with a per-entry index decode longer walks cost more than the
# launches they saved, r06g-r06i)
FUSE = os.environ.get("PGM_FUSE", "1") != "0"
FUSE_BUDGET = int(os.environ.get("PGM_FUSE_BUDGET", 1 << 19))
# reduction entries per output of a fused step
FUSE_MAX_RED = int(os.environ.get("PGM_FUSE_MAX_RED", 512))
# absorb only the inputs on the step's critical path (the deepest): absorbing a shallower one saves no
# level, it only lengthens the job's walk
FUSE_CRITICAL_ONLY = os.environ.get("PGM_FUSE_CRIT", "1") != "0"
FUSE_MAX_OPS = 8   # PGM_PRODN_MAX_OPS
FUSE_MAX_DIMS = 12  # KMAX: kept / reduced dims of one job


def fuse_path(steps, operand_labels, dims, budget=None, max_ops=FUSE_MAX_OPS, max_dims=FUSE_MAX_DIMS, fixed=(),
              max_red=None):
    """A path's pairwise / reduce steps grouped into n-ary steps ("nary", inputs..., keep, nid): walking
    the steps in order, each step absorbs the steps that produced its inputs (deepest first) while the
    group's index space (the union of its inputs' labels) stays within `budget` entries, its inputs
    within `max_ops` and its kept / summed labels within `max_dims` — so C[keep] is the sum over the
    group's other labels of the product of its inputs, the same value as the steps it replaces (every
    intermediate of a path is consumed once).  A group of one step stays that step.  `fixed`: ids of
    steps that keep their own kernel (dense GEMMs, packed reductions): they neither absorb nor are
    absorbed."""
    budget = FUSE_BUDGET if budget is None else budget
    max_red = FUSE_MAX_RED if max_red is None else max_red
    labels = {i: list(dict.fromkeys(ls)) for i, ls in enumerate(operand_labels)}
    depth = {i: 0 for i in labels}
    groups = {}  # nid -> (original step, inputs)
    kept_as_is = set()
    for st in steps:
        ins, keep, nid = list(st[1:-2]), st[-2], st[-1]
        labels[nid] = keep
        if nid in fixed:
            kept_as_is.add(nid)
            depth[nid] = 1 + max(depth[y] for y in ins)
            continue
        cur = list(ins)
        while True:
            done = True
            top = max(depth[y] for y in cur)
            for x in sorted((x for x in cur if x in groups), key=lambda x: -depth[x]):
                if FUSE_CRITICAL_ONLY and depth[x] < top:
                    break
                trial = [y for y in cur if y != x] + groups[x][1]
                space = list(dict.fromkeys(l for y in trial for l in labels[y]))
                n_space = _size(space, dims)
                if (len(trial) <= max_ops and n_space <= budget and len(keep) <= max_dims
                        and len(space) - len(keep) <= max_dims and n_space <= max_red * _size(keep, dims)):
                    cur = trial
                    del groups[x]
                    done = False
                    break
            if done:
                break
        groups[nid] = (st, cur)
        depth[nid] = 1 + max(depth[y] for y in cur)
    out = []
    for st in steps:
        if st[-1] in kept_as_is:
            out.append(st)
            continue
        g = groups.get(st[-1])
        if g is None:
            continue
        orig, cur = g
        out.append(orig if list(cur) == list(orig[1:-2]) else ("nary",) + tuple(cur) + (orig[-2], orig[-1]))
    return out


def plan_stats(operand_labels, out_labels, dims, fuse=False):
    """Algorithmic bytes / flops of the executed path (choose_path, fused as the compiled program runs it
    when `fuse`; SURVEY.md §8(d) C2 definition): sum over steps of 8 (sum |inputs| + |C|) bytes and
    (inputs) x |index space| flops."""
    steps, _ = choose_path(operand_labels, out_labels, dims)
    if fuse:
        steps = fuse_path(steps, operand_labels, dims)
    labels = {i: list(dict.fromkeys(ls)) for i, ls in enumerate(operand_labels)}
    nbytes = flops = 0
    max_inter = sum_inter = 0
    for st in steps:
        ins, keep, nid = st[1:-2], st[-2], st[-1]
        space = list(dict.fromkeys(l for i in ins for l in labels[i]))
        nbytes += 8 * (sum(_size(labels[i], dims) for i in ins) + _size(keep, dims))
        flops += (1 if st[0] == "reduce" else 2 if st[0] == "pair" else len(ins)) * _size(space, dims)
        labels[nid] = keep
        max_inter = max(max_inter, _size(keep, dims))
        sum_inter += _size(keep, dims)
    return {"steps": len(steps), "bytes": nbytes, "flops": flops, "max_intermediate": max_inter,
            "sum_intermediate": sum_inter}


_PATHS = OrderedDict()  # compiled paths, keyed on the operands' (label, cardinality) structure
_PATHS_LOCK = threading.Lock()
PACK_MAX_OUT = 4096       # pack the operands of non-GEMM steps with at most this many outputs ...
PACK_MIN_WORK = 1 << 20   # ... and at least this large an index space
PATH_CACHE_SIZE = 256


def compiled_path(operand_labels, out_labels, dims, order=None, fuse=False):
    """choose_path (or, with `order`, order_path) plus, per pairwise step, the dense-GEMM
    classification (engine.gemm_shape), cached on the contraction's structure: repeated queries with
    the same query / evidence variables (C2's pattern; every row batch of a predict pattern) re-plan
    nothing.  fuse: the steps that are neither GEMMs nor packed grouped into n-ary steps (fuse_path)."""
    key = (tuple(tuple((l, int(dims[l])) for l in ls) for ls in operand_labels), tuple(out_labels),
           None if order is None else tuple(order), bool(fuse))
    with _PATHS_LOCK:  # concurrent queries (engine.device_lock is shared) share this cache
        hit = _PATHS.get(key)
        if hit is not None:
            _PATHS.move_to_end(key)
            return hit
    if order is None:
        steps, final_id = choose_path(operand_labels, out_labels, dims)
    else:
        steps, final_id = order_path(operand_labels, out_labels, dims, order)
    if fuse:
        steps = _fuse_plain(steps, operand_labels, dims)
    labels = {i: list(dict.fromkeys(ls)) for i, ls in enumerate(operand_labels)}
    plan = []
    for st in steps:
        if st[0] in ("reduce", "nary"):
            labels[st[-1]] = st[-2]
            plan.append((st, None))
            continue
        _, i, j, keep, nid = st
        shape = E.gemm_shape(labels[i], labels[j], keep, dims)
        if shape is not None:
            # operand roles and the output layout chosen for coalescing; later steps see that layout
            swap, keep, shape = E.gemm_orient(labels[i], labels[j], shape)
            st = ("pair", j, i, keep, nid) if swap else ("pair", i, j, keep, nid)
        elif _size(keep, dims) <= PACK_MAX_OUT and _size(list(dict.fromkeys(labels[i] + labels[j])), dims) >= PACK_MIN_WORK:
            # a long reduction to few outputs (a batched dot product): both operands are first copied to
            # [kept..., summed...] with the summed variables in one shared order, so the reduction is one
            # contiguous run (lanes + split-K) instead of a strided walk with a digit decode per step
            shape = "pack"
        labels[nid] = keep
        plan.append((st, shape))
    # levels: step k runs at 1 + the deepest level among its inputs (inputs are level 0)
    depth = {i: 0 for i in range(len(operand_labels))}
    levels = []
    for k, (st, _) in enumerate(plan):
        ins = st[1:-2]
        d = 1 + max(depth[i] for i in ins)
        depth[st[-1]] = d
        while len(levels) < d:
            levels.append([])
        levels[d - 1].append(k)
    hit = (plan, final_id, levels)
    with _PATHS_LOCK:
        _PATHS[key] = hit
        if len(_PATHS) > PATH_CACHE_SIZE:
            _PATHS.popitem(last=False)
    return hit


def _specialising():
    """Batches of compiled programs become plan-specialised kernels (hipRTC present, not disabled)."""
    from .. import program as P

    return bool(getattr(P, "BATCH_SPECIALISE", False)) and not os.environ.get("PGM_NO_JIT")


def _fuse_plain(steps, operand_labels, dims):
    """fuse_path over the steps that stay plain contractions: a pairwise step that is a dense GEMM
    (engine.gemm_shape) or a packed long reduction keeps its own kernel, so it never joins a group
    (its index space is beyond the budget anyway; checked here rather than assumed)."""
    labels = {i: list(dict.fromkeys(ls)) for i, ls in enumerate(operand_labels)}
    fixed = set()
    for st in steps:
        if st[0] == "pair":
            _, i, j, keep, nid = st
            if (E.gemm_shape(labels[i], labels[j], keep, dims) is not None or
                    (_size(keep, dims) <= PACK_MAX_OUT and
                     _size(list(dict.fromkeys(labels[i] + labels[j])), dims) >= PACK_MIN_WORK)):
                fixed.add(nid)
        labels[st[-1]] = st[-2]
    return fuse_path(steps, operand_labels, dims, fixed=fixed)


def contract_factors(operands, out_labels, reduce="sum", prog=None, order=None):
    """sum_{labels not in out} prod operands, on the device.

    operands: list of (device tensor, labels).  Returns a tensor over
    out_labels (C-order).  reduce="max" gives the max-product variant.  With a
    pgmpy_amd.program.Program the launches are recorded (buffers preallocated)
    instead of issued.  order: eliminate the labels in this order (order_path)
    instead of the planner's choice."""
    run = prog if prog is not None else E
    if not operands:
        raise ValueError("nothing to contract")
    dims = {}
    for t, ls in operands:
        if len(ls) != t.dim():
            raise ValueError("label count does not match tensor rank")
        for d, l in enumerate(ls):
            c = int(t.shape[d])
            if dims.setdefault(l, c) != c:
                raise ValueError(f"cardinality mismatch for {l!r}")
    for l in out_labels:
        if l not in dims:
            raise ValueError(f"output label {l!r} not in any operand")
    # n-ary fusion for compiled plain programs whose batches become plan-specialised kernels (the only
    # kernels that run n-ary jobs)
    fuse = (FUSE and prog is not None and not getattr(prog, "_levels", True) and _specialising())
    plan, final_id, levels = compiled_path([ls for _, ls in operands], out_labels, dims, order=order, fuse=fuse)
    live = {i: (t, list(ls)) for i, (t, ls) in enumerate(operands)}

    after = []  # contractions that read operands packed in the same level (recorded after its batch)

    def step(st, shape):
        if st[0] == "reduce":
            _, i, keep, nid = st
            t, ls = live.pop(i)
            live[nid] = (run.contract(t, ls, None, None, keep, reduce=reduce, combine="copy"), keep)
        elif st[0] == "nary":
            ins, keep, nid = st[1:-2], st[-2], st[-1]
            live[nid] = (prog.contract_n([live.pop(i) for i in ins], keep, reduce=reduce), keep)
        else:
            _, i, j, keep, nid = st
            ti, li = live.pop(i)
            tj, lj = live.pop(j)
            if shape == "pack":
                red = [l for l in dict.fromkeys(li + lj) if l not in keep]
                pa = [l for l in keep if l in li] + [l for l in red if l in li]
                pb = [l for l in keep if l in lj] + [l for l in red if l in lj]
                ti, li = run.contract(ti, li, None, None, pa, combine="copy"), pa
                tj, lj = run.contract(tj, lj, None, None, pb, combine="copy"), pb
                if prog is None:
                    live[nid] = (E.contract(ti, li, tj, lj, keep, reduce=reduce, combine="mul"), keep)
                else:
                    after.append((nid, ti, li, tj, lj, keep))
            elif shape is not None and reduce == "sum":
                live[nid] = ((prog.pair_gemm(ti, li, tj, lj, keep, shape) if prog is not None
                              else E.pair_gemm(ti, li, tj, lj, keep, shape=shape)), keep)
            else:
                live[nid] = (run.contract(ti, li, tj, lj, keep, reduce=reduce, combine="mul"), keep)

    if prog is None:
        for st, shape in plan:
            step(st, shape)
    else:
        # recorded: one launch per level of the path (steps whose inputs are all ready); a packed
        # step's contraction follows its level's batch (it reads the copies made inside it)
        for lvl in levels:
            prog.begin_batch()
            for k in lvl:
                step(*plan[k])
            prog.end_batch()
            for nid, ti, li, tj, lj, keep in after:
                live[nid] = (prog.contract(ti, li, tj, lj, keep, reduce=reduce, combine="mul"), keep)
            after.clear()
    t, ls = live[final_id]
    if ls != list(out_labels):
        t = run.contract(t, ls, None, None, list(out_labels), reduce=reduce, combine="copy")
    return t
