"""Offline stand-in for ``opt_einsum.contract`` (fixture generation only).

The reference calls ``opt_einsum.contract(*[arr, labels]*, out_labels,
optimize="greedy")`` (pgmpy/inference/ExactInference.py:404-406,
pgmpy/factors/base.py:106).  opt_einsum is not installed in this image, so this
module restates its *greedy* strategy: sum private indices first, then
repeatedly contract the pair of operands with the smallest
``size(out) - size(a) - size(b)`` (pairs that share an index first), keeping an
index while any other operand or the output still needs it.  Contraction
values do not depend on the path beyond floating-point rounding.
"""
import string

import numpy as np

__version__ = "0.0-shim"

_LETTERS = string.ascii_letters


def _size(labels, dims):
    s = 1
    for l in labels:
        s *= dims[l]
    return s


def _einsum_local(ops, out):
    """np.einsum with labels relabelled to letters (np sublists need < 52 labels)."""
    lab = {}
    for _, ls in ops:
        for l in ls:
            if l not in lab:
                lab[l] = _LETTERS[len(lab)]
    for l in out:
        if l not in lab:
            lab[l] = _LETTERS[len(lab)]
    expr = ",".join("".join(lab[l] for l in ls) for _, ls in ops) + "->" + "".join(lab[l] for l in out)
    return np.einsum(expr, *[a for a, _ in ops])


def contract(*args, optimize="greedy", **kwargs):
    args = list(args)
    out_labels = list(args[-1])
    args = args[:-1]
    ops = []
    for i in range(0, len(args), 2):
        ops.append((np.asarray(args[i]), list(args[i + 1])))
    dims = {}
    for a, ls in ops:
        for d, l in zip(a.shape, ls):
            dims[l] = d
    if not ops:
        return np.array(1.0)

    def needed_elsewhere(label, skip):
        if label in out_labels:
            return True
        for j, (_, ls) in enumerate(ops):
            if j in skip:
                continue
            if label in ls:
                return True
        return False

    # private index reduction (and dedupe repeated labels)
    new_ops = []
    for i, (a, ls) in enumerate(ops):
        keep = []
        for l in ls:
            if l in keep:
                continue
            if needed_elsewhere(l, {i}):
                keep.append(l)
        if keep != ls:
            a = _einsum_local([(a, ls)], keep)
        new_ops.append((a, keep))
    ops = new_ops

    # heap of candidate pairs that share a label (lazy deletion of dead operands)
    import heapq

    live = {i: op for i, op in enumerate(ops)}
    holders = {}
    for i, (_, ls) in live.items():
        for l in ls:
            holders.setdefault(l, set()).add(i)
    nxt = len(ops)

    def kept(labels, exclude):
        return [l for l in labels if l in out_labels or len(holders[l] - exclude) > 0]

    heap, seen = [], set()

    def push(i):
        partners = set()
        for l in live[i][1]:
            partners |= holders[l]
        partners.discard(i)
        for j in partners:
            key = (min(i, j), max(i, j))
            if key in seen:
                continue
            seen.add(key)
            li, lj = live[key[0]][1], live[key[1]][1]
            keep = kept(list(dict.fromkeys(li + lj)), set(key))
            cost = _size(keep, dims) - _size(li, dims) - _size(lj, dims)
            heapq.heappush(heap, (cost, key[0], key[1], keep))

    for i in list(live):
        push(i)
    while len(live) > 1:
        pick = None
        while heap:
            cost, a, b, keep = heapq.heappop(heap)
            if a in live and b in live:
                pick = (a, b, keep)
                break
        if pick is None:
            a, b = sorted(live, key=lambda k: (_size(live[k][1], dims), k))[:2]
            pick = (a, b, kept(list(dict.fromkeys(live[a][1] + live[b][1])), {a, b}))
        a, b, keep = pick
        res = _einsum_local([live[a], live[b]], keep)
        for l in live[a][1] + live[b][1]:
            holders[l].discard(a)
            holders[l].discard(b)
        del live[a], live[b]
        nid = nxt
        nxt += 1
        live[nid] = (res, keep)
        for l in keep:
            holders[l].add(nid)
        push(nid)
    ops = list(live.values())

    a, ls = ops[0]
    return _einsum_local([(a, ls)], out_labels)
