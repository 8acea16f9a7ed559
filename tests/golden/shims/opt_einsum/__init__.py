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

    while len(ops) > 1:
        best = None
        for i in range(len(ops)):
            for j in range(i + 1, len(ops)):
                li, lj = ops[i][1], ops[j][1]
                shared = set(li) & set(lj)
                union = list(dict.fromkeys(li + lj))
                keep = [l for l in union if needed_elsewhere(l, {i, j})]
                cost = _size(keep, dims) - _size(li, dims) - _size(lj, dims)
                key = (0 if shared else 1, cost)
                if best is None or key < best[0]:
                    best = (key, i, j, keep)
        _, i, j, keep = best
        res = _einsum_local([ops[i], ops[j]], keep)
        ops = [op for k, op in enumerate(ops) if k not in (i, j)] + [(res, keep)]

    a, ls = ops[0]
    return _einsum_local([(a, ls)], out_labels)
