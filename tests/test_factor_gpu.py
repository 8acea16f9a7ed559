"""DiscreteFactor / TabularCPD on the device vs the reference's golden vectors.

Mirrors the reference's hot-path unit tests (test_Factor.py:390-765:
marginalize, normalize, reduce, product/factor_product, divide incl. x/0 = inf,
sum, maximize) on 40 seeded factor pairs whose expected outputs were produced
by pgmpy 1.0.0 (tests/golden/factor_ops.json).  Comparisons are
order-invariant (the reference orders product() outputs by set hash).
Tolerance 1e-12 (fp64; exact for reduce / maximize).
"""
import numpy as np
import pytest

from tests.goldens import aligned, fac_values, load_json

pytestmark = pytest.mark.gpu


def _f(fj):
    from pgmpy_amd.factors.discrete import DiscreteFactor

    return DiscreteFactor(fj["variables"], fj["cardinality"], fac_values(fj))


def _check(phi, fj, exact=False):
    assert set(phi.variables) == set(fj["variables"])
    got = aligned(np.asarray(phi.values), phi.variables, fj["variables"])
    exp = fac_values(fj)
    if exact:
        np.testing.assert_array_equal(got, exp)
    else:
        np.testing.assert_allclose(got, exp, rtol=1e-12, atol=1e-15)


def test_factor_ops_golden(gpu):
    from pgmpy_amd.factors import factor_product

    g = load_json("factor_ops.json")
    for c in g["cases"]:
        a, b = _f(c["a"]), _f(c["b"])
        _check(a.product(b, inplace=False), c["product"])
        _check(a * b, c["product"])
        _check(a.sum(b, inplace=False), c["sum"])
        _check(a.marginalize(c["marg_vars"], inplace=False), c["marginalize"])
        _check(a.maximize(c["marg_vars"], inplace=False), c["maximize"], exact=True)
        _check(a.normalize(inplace=False), c["normalize"])
        _check(a.reduce([tuple(x) for x in c["reduce_vals"]], inplace=False), c["reduce"], exact=True)
        _check(a.divide(_f(c["den"]), inplace=False), c["divide"])
        _check(factor_product(a, b, _f(c["c"])), c["factor_product3"])
        # in-place variants mutate and return None
        a2 = _f(c["a"])
        assert a2.marginalize(c["marg_vars"]) is None
        _check(a2, c["marginalize"])


def test_unit_cases(gpu):
    from pgmpy_amd.factors.discrete import DiscreteFactor, TabularCPD

    u = load_json("unit_cases.json")
    phi = DiscreteFactor(["x1", "x2", "x3"], [2, 3, 2], range(12))
    phi.marginalize(["x1", "x3"])
    _check(phi, u["marg_x1_x3"])
    phi1 = DiscreteFactor(["x1", "x2", "x3"], [2, 3, 2], range(12))
    phi2 = DiscreteFactor(["x3", "x4", "x1"], [2, 2, 2], range(8))
    _check(phi1.product(phi2, inplace=False), u["product_doc"])
    _check(phi1.sum(phi2, inplace=False), u["sum_doc"])
    _check(phi1.divide(DiscreteFactor(["x3", "x1"], [2, 2], range(1, 5)), inplace=False), u["divide_doc"])
    num = DiscreteFactor(["x1", "x2"], [2, 2], [0.0, 1.0, 2.0, 0.0])
    r = num.divide(DiscreteFactor(["x1"], [2], [0.0, 2.0]), inplace=False)
    np.testing.assert_array_equal(aligned(r.values, r.variables, u["divide_zero"]["variables"]),
                                  fac_values(u["divide_zero"]))
    mx = DiscreteFactor(["x1", "x2", "x3"], [3, 2, 2],
                        [0.25, 0.35, 0.08, 0.16, 0.05, 0.07, 0.00, 0.00, 0.15, 0.21, 0.09, 0.18])
    _check(mx.maximize(["x2"], inplace=False), u["maximize_doc"], exact=True)
    cpd = TabularCPD("grade", 2, [[0.7, 0.2, 0.6, 0.2], [0.4, 0.4, 0.4, 0.8]], ["intel", "diff"], [2, 2])
    np.testing.assert_allclose(cpd.normalize(inplace=False).get_values(), u["cpd_normalize"], rtol=1e-12)
    cpd2 = TabularCPD("grade", 2, [[0.7, 0.6, 0.6, 0.2], [0.3, 0.4, 0.4, 0.8]], ["intel", "diff"], [2, 2])
    np.testing.assert_allclose(cpd2.marginalize(["diff"], inplace=False).get_values(), u["cpd_marginalize_diff"],
                               rtol=1e-12)
    np.testing.assert_allclose(cpd2.reduce([("diff", 0)], inplace=False).get_values(), u["cpd_reduce_diff0"],
                               rtol=1e-12)


def test_errors_match_reference(gpu):
    """Exception types of test_Factor.py (TypeError / ValueError / IndexError)."""
    from pgmpy_amd.factors.discrete import DiscreteFactor

    phi = DiscreteFactor(["x1", "x2", "x3"], [2, 3, 2], range(12))
    with pytest.raises(TypeError):
        phi.marginalize("x1")
    with pytest.raises(ValueError):
        phi.marginalize(["x9"])
    with pytest.raises(IndexError):
        phi.reduce([("x1", 5)])
    with pytest.raises(ValueError):
        phi.divide(DiscreteFactor(["x9"], [2], [1, 2]))
    with pytest.raises(TypeError):
        DiscreteFactor("x1", [2], [1, 2])
    with pytest.raises(ValueError):
        DiscreteFactor(["x1"], [2], [1, 2, 3])


def test_state_names_and_eq(gpu):
    from pgmpy_amd.factors.discrete import DiscreteFactor

    sn = {"speed": ["low", "medium", "high"], "switch": ["on", "off"]}
    phi = DiscreteFactor(["speed", "switch"], [3, 2], np.arange(6), state_names=sn)
    r = phi.reduce([("speed", "medium")], inplace=False)
    np.testing.assert_array_equal(r.values, [2.0, 3.0])
    assert r.state_names == {"switch": ["on", "off"]}
    phi_t = DiscreteFactor(["switch", "speed"], [2, 3], np.arange(6).reshape(3, 2).T.ravel(), state_names=sn)
    assert phi == phi_t
    assert phi.assignment([1, 5]) == [[("speed", "low"), ("switch", "off")], [("speed", "high"), ("switch", "off")]]
    # host edits of .values are honoured by the next device op
    v = phi.values
    v[0, 0] = 100.0
    assert float(phi.marginalize(["switch"], inplace=False).values[0]) == 101.0


def test_large_factor_ops(gpu):
    """Multi-million-entry factors (munin-size cliques, SURVEY.md §8 table: 2.74M states)."""
    from pgmpy_amd.factors.discrete import DiscreteFactor

    rng = np.random.default_rng(3)
    a = rng.random((14, 14, 14, 10, 10, 10))
    b = rng.random((10, 14, 21))
    A = DiscreteFactor(["a", "b", "c", "d", "e", "f"], a.shape, a)
    B = DiscreteFactor(["f", "c", "g"], b.shape, b)
    P = A.product(B, inplace=False)
    ref = np.einsum("abcdef,fcg->abcdefg", a, b)
    np.testing.assert_allclose(aligned(P.values, P.variables, list("abcdefg")), ref, rtol=1e-14)
    M = A.marginalize(["b", "d", "f"], inplace=False)
    np.testing.assert_allclose(M.values, a.sum(axis=(1, 3, 5)), rtol=1e-11)
    N = A.normalize(inplace=False)
    np.testing.assert_allclose(N.values, a / a.sum(), rtol=1e-11)


def test_api_extras_against_reference(gpu):
    """VERDICT r05 #8 against the reference's own outputs (make_golden.py gen_api_extras):
    DiscreteBayesianNetwork.get_state_probability (DiscreteBayesianNetwork.py:991-1041; asia incl. the
    docstring's 0.02605122, alarm with 31 and 37 of 37 variables assigned) through the device contraction,
    its ValueErrors; TabularCPD.reorder_parents (CPD.py:598-727) inplace and not, on the docstring CPD and
    alarm's CATECHOL, including the reference's reset of the state names when inplace; to_dataframe
    (CPD.py:336-410) on three alarm CPDs."""
    import pandas as pd

    from pgmpy_amd.factors.discrete import TabularCPD
    from pgmpy_amd.utils import get_example_model

    g = load_json("api_extras.json")
    nets = {n: get_example_model(n) for n in ("asia", "alarm")}
    for c in g["state_probability"]:
        got = nets[c["network"]].get_state_probability(c["states"])
        np.testing.assert_allclose(got, c["probability"], rtol=1e-12, atol=1e-300, err_msg=str(c["states"]))
    for e in g["state_probability_errors"]:
        with pytest.raises(ValueError, match=e["message"].split(":")[0]):
            nets["asia"].get_state_probability(e["states"])
    alarm = nets["alarm"]
    for c in g["reorder_parents"]:
        b = c["cpd"]
        sn = {k: list(v) for k, v in b["state_names"].items()}
        cpd = TabularCPD(b["variable"], b["variable_card"], b["values"], b["evidence"], b["evidence_card"],
                         state_names=sn if b["variable"] != "grade" else {})
        r = cpd.reorder_parents(c["new_order"], inplace=c["inplace"])
        np.testing.assert_array_equal(np.asarray(r), np.asarray(c["returned"]))
        assert list(cpd.variables) == c["variables_after"]
        assert [int(x) for x in cpd.cardinality] == c["cardinality_after"]
        np.testing.assert_array_equal(np.asarray(cpd.values).ravel(), np.asarray(c["values_after"]))
        assert {k: [str(x) for x in v] for k, v in cpd.state_names.items()} == c["state_names_after"]
    with pytest.raises(ValueError, match="New order either has missing or extra arguments"):
        TabularCPD("grade", 3, [[0.1] * 6, [0.3] * 6, [0.6] * 6], ["diff", "intel"], [2, 3]).reorder_parents(["intel"])
    for c in g["to_dataframe"]:
        df = alarm.get_cpds(c["node"]).to_dataframe()
        assert isinstance(df, pd.DataFrame)
        assert [str(x) for x in df.columns] == c["columns"] and str(df.columns.name) == c["columns_name"]
        assert [str(n) for n in df.index.names] == c["index_names"]
        assert [[str(x) for x in (t if isinstance(t, tuple) else (t,))] for t in df.index] == c["index"]
        np.testing.assert_array_equal(df.to_numpy(), np.asarray(c["values"]))
