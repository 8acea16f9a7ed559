"""numpy restatement of DiscreteFactor algebra (ORACLE — test infrastructure only).

Follows pgmpy/factors/discrete/DiscreteFactor.py: marginalize L360-411,
maximize L413-483, normalize L485-533, reduce L535-617, sum L619-715,
product L717-792, divide L794-866.  Variable order of products is the
deterministic union (self vars then new ones) instead of the reference's
set-hash order; comparisons are order-invariant (aligned()).
"""
import numpy as np


class OFactor:
    __slots__ = ("vars", "card", "values")

    def __init__(self, variables, cardinality, values):
        self.vars = list(variables)
        self.card = [int(c) for c in cardinality]
        self.values = np.asarray(values, dtype=np.float64).reshape(self.card)

    def copy(self):
        return OFactor(self.vars, self.card, self.values.copy())

    def aligned(self, order):
        """values transposed to `order` (order-invariant comparison)."""
        return np.transpose(self.values, [self.vars.index(v) for v in order]) if self.vars else self.values

    # DiscreteFactor.py:717-792 — einsum broadcast product, no summed index
    def product(self, other):
        if np.isscalar(other):
            return OFactor(self.vars, self.card, self.values * other)
        union = self.vars + [v for v in other.vars if v not in self.vars]
        lab = {v: i for i, v in enumerate(union)}
        vals = np.einsum(self.values, [lab[v] for v in self.vars], other.values, [lab[v] for v in other.vars],
                         list(range(len(union))))
        card = {**dict(zip(self.vars, self.card)), **dict(zip(other.vars, other.card))}
        return OFactor(union, [card[v] for v in union], vals)

    # DiscreteFactor.py:360-411 — einsum sum over the listed axes
    def marginalize(self, variables):
        for v in variables:
            if v not in self.vars:
                raise ValueError(f"{v} not in scope.")
        keep = [i for i, v in enumerate(self.vars) if v not in variables]
        vals = np.einsum(self.values, list(range(len(self.vars))), keep)
        return OFactor([self.vars[i] for i in keep], [self.card[i] for i in keep], vals)

    # DiscreteFactor.py:413-483 — np.max over axes
    def maximize(self, variables):
        axes = tuple(self.vars.index(v) for v in variables)
        keep = [i for i in range(len(self.vars)) if i not in axes]
        return OFactor([self.vars[i] for i in keep], [self.card[i] for i in keep], np.max(self.values, axis=axes))

    # DiscreteFactor.py:485-533 — values / values.sum(), 0/0 -> NaN kept
    def normalize(self):
        with np.errstate(invalid="ignore", divide="ignore"):
            return OFactor(self.vars, self.card, self.values / self.values.sum())

    # DiscreteFactor.py:535-617 — basic indexing by state numbers
    def reduce(self, assignment):
        sl = [slice(None)] * len(self.vars)
        for v, s in assignment.items():
            sl[self.vars.index(v)] = s
        keep = [i for i, v in enumerate(self.vars) if v not in assignment]
        return OFactor([self.vars[i] for i in keep], [self.card[i] for i in keep], self.values[tuple(sl)])

    # DiscreteFactor.py:619-715 — broadcast add, new variables appended
    def sum(self, other):
        if np.isscalar(other):
            return OFactor(self.vars, self.card, self.values + other)
        union = self.vars + [v for v in other.vars if v not in self.vars]
        card = {**dict(zip(self.vars, self.card)), **dict(zip(other.vars, other.card))}
        a = self.values.reshape(self.card + [1] * (len(union) - len(self.vars)))
        b = _broadcast_to(other, union, card)
        return OFactor(union, [card[v] for v in union], a + b)

    # DiscreteFactor.py:794-866 — broadcast divide, NaN -> 0
    def divide(self, other):
        if set(other.vars) - set(self.vars):
            raise ValueError("Scope of divisor should be a subset of dividend")
        card = dict(zip(self.vars, self.card))
        b = _broadcast_to(other, self.vars, card)
        with np.errstate(invalid="ignore", divide="ignore"):
            v = self.values / b
        v[np.isnan(v)] = 0
        return OFactor(self.vars, self.card, v)


def _broadcast_to(f, order, card):
    present = [v for v in order if v in f.vars]
    vals = f.aligned(present)
    shape = [card[v] if v in f.vars else 1 for v in order]
    return vals.reshape(shape)


def product_all(factors):
    out = factors[0]
    for f in factors[1:]:
        out = out.product(f)
    return out
