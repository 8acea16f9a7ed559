"""The "hip" backend at pgmpy's own operator seam (pgmpy_amd.compat) against the reference goldens.

pgmpy with ``config.set_backend("hip")`` would hold ``DiscreteFactor.values`` as HipArray and call
``compat_fns`` / plain array arithmetic exactly as its numpy path does.  `SeamFactor` below performs
those calls in the reference's order for each hot-path method — marginalize (einsum sublist,
DiscreteFactor.py:408), maximize (compat_fns.max, L480), normalize (values / values.sum(), L530),
reduce (basic indexing, L614), sum (np.newaxis + swapaxes + add, L690-712), product (scalar *=,
L765-766; two-operand einsum, L771-777), divide (newaxis + swapaxes + "/" + values[isnan] = 0,
L835-863) and map_query's argmax (ExactInference.py:616) — through pgmpy_amd.compat only, and
the results are compared with the outputs pgmpy 1.0.0 produced (tests/golden/factor_ops.json).
"""
import numpy as np
import pytest

from tests.goldens import aligned, fac_values, load_json

pytestmark = pytest.mark.gpu


class SeamFactor:
    """The reference's call sequence per method over compat (variables / cardinality on the host,
    values a HipArray)."""

    def __init__(self, variables, cardinality, values):
        from pgmpy_amd import compat

        self.C = compat
        self.variables = list(variables)
        self.cardinality = np.array(cardinality, dtype=int)
        self.values = compat.values_array(values, cardinality)

    def _clone(self):
        f = SeamFactor.__new__(SeamFactor)
        f.C, f.variables, f.cardinality = self.C, list(self.variables), self.cardinality.copy()
        f.values = self.C.copy(self.values)
        return f

    def marginalize(self, names):
        f = self._clone()
        drop = [f.variables.index(v) for v in names]
        keep = sorted(set(range(len(f.variables))) - set(drop))
        f.values = self.C.einsum(f.values, range(len(f.variables)), keep)
        f.variables = [f.variables[i] for i in keep]
        return f

    def maximize(self, names):
        f = self._clone()
        drop = [f.variables.index(v) for v in names]
        keep = sorted(set(range(len(f.variables))) - set(drop))
        f.values = self.C.max(f.values, axis=tuple(drop))
        f.variables = [f.variables[i] for i in keep]
        return f

    def normalize(self):
        f = self._clone()
        f.values = f.values / (f.values.sum())
        return f

    def reduce(self, pairs):
        f = self._clone()
        idx = [slice(None)] * len(f.variables)
        gone = []
        for v, s in pairs:
            i = f.variables.index(v)
            idx[i] = s
            gone.append(i)
        f.values = f.values[tuple(idx)]
        f.variables = [v for i, v in enumerate(f.variables) if i not in gone]
        return f

    def _aligned_operand(self, other):
        """other's values with extra axes (np.newaxis) and axes swapped into self's order."""
        vals, names = other.values, list(other.variables)
        extra = [v for v in self.variables if v not in names]
        if extra:
            vals = vals[tuple([slice(None)] * len(names) + [None] * len(extra))]
            names += extra
        for axis in range(len(self.variables)):
            j = names.index(self.variables[axis])
            names[axis], names[j] = names[j], names[axis]
            vals = vals.swapaxes(axis, j)
        return vals

    def sum(self, other):
        f = self._clone()
        new = [v for v in other.variables if v not in f.variables]
        if new:  # the reference first extends self with other's extra variables (L677-688)
            f.values = f.values[tuple([slice(None)] * len(f.variables) + [None] * len(new))]
            card = dict(zip(other.variables, other.cardinality))
            f.variables += new
            f.cardinality = np.append(f.cardinality, [card[v] for v in new])
        f.values = f.values + f._aligned_operand(other)
        return f

    def product(self, other):
        f = self._clone()
        if isinstance(other, (int, float)):
            f.values *= other
            return f
        union = list(dict.fromkeys(f.variables + other.variables))
        pos = {v: i for i, v in enumerate(union)}
        f.values = self.C.einsum(f.values, [pos[v] for v in f.variables], other.values,
                                 [pos[v] for v in other.variables], range(len(union)))
        f.variables = union
        return f

    def divide(self, other):
        f = self._clone()
        f.values = f.values / f._aligned_operand(other)
        f.values[self.C.get_compute_backend().isnan(f.values)] = 0
        return f


def _check(f, fj, exact=False):
    assert set(f.variables) == set(fj["variables"])
    got = aligned(np.asarray(f.values), f.variables, fj["variables"])
    if exact:
        np.testing.assert_array_equal(got, fac_values(fj))
    else:
        np.testing.assert_allclose(got, fac_values(fj), rtol=1e-12, atol=1e-15)


def test_hip_backend_seam_replays_reference_call_shapes(gpu):
    from pgmpy_amd import compat

    compat.config.set_backend("hip")
    try:
        g = load_json("factor_ops.json")
        for c in g["cases"]:
            a = SeamFactor(c["a"]["variables"], c["a"]["cardinality"], fac_values(c["a"]))
            b = SeamFactor(c["b"]["variables"], c["b"]["cardinality"], fac_values(c["b"]))
            den = SeamFactor(c["den"]["variables"], c["den"]["cardinality"], fac_values(c["den"]))
            _check(a.product(b), c["product"])
            _check(a.sum(b), c["sum"])
            _check(a.marginalize(c["marg_vars"]), c["marginalize"])
            _check(a.maximize(c["marg_vars"]), c["maximize"], exact=True)
            _check(a.normalize(), c["normalize"])
            _check(a.reduce([tuple(x) for x in c["reduce_vals"]]), c["reduce"], exact=True)
            _check(a.divide(den), c["divide"])
            # scalar product (L765-766) and map_query's argmax (ExactInference.py:616)
            np.testing.assert_allclose(np.asarray(a.product(2.5).values), 2.5 * fac_values(c["a"]), rtol=1e-15)
            assert compat.argmax(a.values) == int(np.argmax(fac_values(c["a"])))
    finally:
        compat.config.set_backend("numpy")


def test_hip_backend_assignment_eq_valid_cpd_and_totals(gpu):
    """The rest of the seam pgmpy calls on a non-numpy backend, in the reference's order:
    assignment (DiscreteFactor.py:290-320: torch index, get_compute_backend().zeros, % and //,
    compat_fns.flip), __eq__ (L1079: compat_fns.allclose), is_valid_cpd (L959-964:
    get_compute_backend().allclose of values.flatten() and compat_fns.ones), the partition function
    (DiscreteMarkovNetwork.py:844: compat_fns.sum), the virtual-evidence CPD (inference/base.py:286:
    get_compute_backend().vstack of values and 1 - values), sampling's unique (sampling/base.py:148)
    and exp (MirrorDescentEstimator.py:88)."""
    import torch

    from pgmpy_amd import compat

    compat.config.set_backend("hip")
    try:
        card = np.array([2, 3, 2])
        vals = np.arange(12, dtype=np.float64)
        values = compat.values_array(vals, card)
        # assignment([1, 7, 11]) as DiscreteFactor.assignment runs it on a non-numpy backend
        index = torch.tensor([1, 7, 11], dtype=torch.int, device=compat.config.get_device())
        assignments = compat.get_compute_backend().zeros((len(index), 3), dtype=int)
        for i, c in enumerate(card[::-1]):
            assignments[:, i] = index % int(c)
            index = index // int(c)
        assignments = compat.flip(assignments, axis=(1,))
        got = [[int(v) for v in row] for row in assignments]
        exp_rows = [list(np.unravel_index(k, card)) for k in (1, 7, 11)]
        assert got == [[int(x) for x in r] for r in exp_rows]
        # __eq__ / is_valid_cpd
        assert compat.allclose(values, compat.values_array(vals + 1e-9, card), atol=1e-8)
        assert not compat.allclose(values, compat.values_array(vals + 1e-3, card), atol=1e-8)
        cpd = compat.values_array(np.array([[0.2, 0.7, 0.5], [0.8, 0.3, 0.5]]), (2, 3))
        col_sums = compat.einsum(cpd, range(2), [1])
        assert compat.get_compute_backend().allclose(col_sums.flatten(), compat.ones(3), atol=0.01)
        # partition function, virtual evidence CPD, unique, exp
        assert compat.sum(values) == pytest.approx(66.0, rel=1e-15)
        ve = compat.values_array(np.array([0.3, 0.7]), (2,))
        stacked = compat.get_compute_backend().vstack((ve, 1 - ve))
        np.testing.assert_allclose(np.asarray(stacked), [[0.3, 0.7], [0.7, 0.3]], rtol=1e-15)
        u, counts = compat.unique(compat.values_array(np.array([2.0, 1.0, 2.0]), (3,)), return_counts=True)
        assert list(u) == [1.0, 2.0] and list(counts) == [1, 2]
        np.testing.assert_allclose(np.asarray(compat.exp(ve)), np.exp([0.3, 0.7]), rtol=1e-15)
    finally:
        compat.config.set_backend("numpy")


def test_hip_backend_divide_zero_and_index_errors(gpu):
    """divide keeps x/0 = inf and maps 0/0 to 0 (the reference's divide_zero fixture); an
    out-of-range state raises IndexError (test_Factor.py:555-565)."""
    from pgmpy_amd import compat

    u = load_json("unit_cases.json")
    compat.config.set_backend("hip")
    try:
        num = SeamFactor(["x1", "x2"], [2, 2], [0.0, 1.0, 2.0, 0.0])
        r = num.divide(SeamFactor(["x1"], [2], [0.0, 2.0]))
        np.testing.assert_array_equal(aligned(np.asarray(r.values), r.variables, u["divide_zero"]["variables"]),
                                      fac_values(u["divide_zero"]))
        with pytest.raises(IndexError):
            num.reduce([("x1", 5)])
        assert compat.size(num.values) == 4 and compat.tobytes(num.values) == np.asarray(num.values).tobytes()
        np.testing.assert_array_equal(compat.ravel_f(num.values), np.array([[0.0, 1.0], [2.0, 0.0]]).ravel("F"))
    finally:
        compat.config.set_backend("numpy")
