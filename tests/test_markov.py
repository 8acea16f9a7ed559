"""DiscreteMarkovNetwork / ClusterGraph / JunctionTree containers and inference over Markov networks.

Goldens: tests/golden/markov_cases.json, written by running the reference (make_golden.py
gen_markov): the moralised 6-node network of test_ExactInference.py:659-889 (SAMIAM values), the
duplicated-factor case (L639-656), the 4-cycle of test_DiscreteMarkovNetwork.py:246-591, a seeded
12-variable pairwise + triangle network and alarm.to_markov_model().

CPU tests pin the oracle (oracle/markov.py) and the host-side structure code (triangulation,
check_model, conversions); `-m gpu` tests run VariableElimination / BeliefPropagation over the
Markov networks through the HIP library and compare with the goldens.
Tolerances: 1e-12 absolute (+1e-10 relative) on potentials and probabilities (fp64).
"""
import numpy as np
import pytest

from oracle import markov as OM
from oracle.factor import OFactor
from tests.goldens import aligned, fac_values, load_json

G = load_json("markov_cases.json")
CASES = ("markov6", "cycle4", "random12")
# random12's heuristic scores tie; the reference breaks ties by string-hash set order, so its H6
# junction tree is pinned only where the cliques coincide
TIE_FREE = ("markov6", "cycle4")


def _ofactors(case):
    return [OFactor(f["variables"], f["cardinality"], fac_values(f)) for f in case["factors"]]


def _card(case):
    card = {}
    for f in case["factors"]:
        card.update(zip(f["variables"], f["cardinality"]))
    return card


def _model(case):
    from pgmpy_amd.factors.discrete import DiscreteFactor
    from pgmpy_amd.models import DiscreteMarkovNetwork

    mm = DiscreteMarkovNetwork([tuple(e) for e in case["edges"]])
    mm.add_factors(*[DiscreteFactor(f["variables"], f["cardinality"], fac_values(f)) for f in case["factors"]])
    return mm


def _close(got, fj, order=None, atol=1e-12):
    exp = fac_values(fj)
    if order is not None:
        exp = aligned(exp, fj["variables"], order)
    np.testing.assert_allclose(np.asarray(got, dtype=np.float64).reshape(exp.shape), exp, rtol=1e-10, atol=atol)


def _values(phi, order):
    return np.transpose(np.asarray(phi.values), [phi.variables.index(v) for v in order])


# ----------------------------------------------------------------------------- oracle pinning (CPU)
@pytest.mark.parametrize("name", CASES)
def test_oracle_markov_against_reference(name):
    case = G[name]
    facs = _ofactors(case)
    states = {v: [str(i) for i in range(c)] for v, c in _card(case).items()}
    for q in case["queries"]:
        ev = {k: int(v) for k, v in q["evidence"].items()}
        _close(OM.query(facs, q["variables"], ev), q["joint"], q["variables"])
        for v, fj in q["separate"].items():
            _close(OM.query(facs, [v], ev), fj)
    for m in case["maps"]:
        got = OM.map_query(facs, m["variables"], {k: int(v) for k, v in m["evidence"].items()}, states)
        assert got == m["result"]
    for m in case["max_marginals"]:
        ev = {k: int(v) for k, v in (m["evidence"] or {}).items()}
        assert OM.max_marginal(facs, m["variables"], ev) == pytest.approx(m["result"], rel=1e-12)
    assert OM.partition(facs) == pytest.approx(case["partition_function"], rel=1e-12)
    card = _card(case)
    edges = [tuple(e) for e in case["edges"]]
    for h, exp in case.get("triangulations", {}).items():
        assert OM.triangulate(edges, card, h) == exp, h
    if name in TIE_FREE:
        assert OM.jt_cliques(edges, card) == case["jt_cliques"]
    beliefs, seps = OM.calibrate(facs, [tuple(c) for c in case["jt_cliques"]], card)
    for c, fj in case["bp_clique_beliefs"]:
        _close(beliefs[tuple(c)].aligned(c), fj)
    mx, _ = OM.calibrate(facs, [tuple(c) for c in case["jt_cliques"]], card, op="max")
    for c, fj in case["bp_max_clique_beliefs"]:
        _close(mx[tuple(c)].aligned(c), fj)


def test_oracle_duplicated_and_alarm_markov():
    d = G["duplicated"]
    facs = [OFactor(f["variables"], f["cardinality"], fac_values(f)) for f in d["factors"]]
    _close(OM.query(facs, ["A"], {}), d["query_A"])
    from oracle.network import load_network

    net = load_network("alarm")
    facs = [net.factor(v) for v in net.nodes]
    for q in G["alarm_markov"]["queries"]:
        ev = {v: net.state_no(v, s) for v, s in q["evidence"].items()}
        _close(OM.query(facs, q["variables"], ev), q["joint"], q["variables"], atol=1e-14)


# ----------------------------------------------------------------------------- host structure (CPU)
@pytest.mark.parametrize("name", CASES)
def test_triangulation_heuristics_match_reference(name):
    import networkx as nx

    case = G[name]
    mm = _model(case)
    for h, exp in case.get("triangulations", {}).items():
        tri = mm.triangulate(heuristic=h)
        assert sorted(sorted(e) for e in tri.edges()) == exp, h
        assert tri.is_triangulated()
    if "order_triangulation" in case:
        t = case["order_triangulation"]
        assert sorted(sorted(e) for e in mm.triangulate(order=t["order"]).edges()) == t["edges"]
    card = _card(case)
    edges = [tuple(e) for e in case["edges"]]
    cl = sorted(sorted(c) for c in nx.find_cliques(mm.triangulate()))
    assert cl == OM.jt_cliques(edges, card)  # same scores, same tie rule as the oracle
    if name in TIE_FREE:
        assert cl == case["jt_cliques"]


def test_triangulate_inplace_and_order():
    mm = _model(G["cycle4"])
    h = mm.triangulate(heuristic="H1", inplace=True)
    assert h is mm and mm.is_triangulated()
    assert sorted(sorted(e) for e in mm.edges()) == G["cycle4"]["triangulations"]["H1"]
    mm2 = _model(G["cycle4"])
    tri = mm2.triangulate(order=["b", "a", "c", "d"])
    assert sorted(sorted(e) for e in tri.edges()) == [["a", "b"], ["a", "c"], ["a", "d"], ["b", "c"], ["c", "d"]]
    assert mm2.triangulate() is not mm2 and not mm2.is_triangulated()


def test_markov_container_semantics():
    """test_DiscreteMarkovNetwork.py:13-405 (creation, cardinality, check_model, factors)."""
    from pgmpy_amd.factors.discrete import DiscreteFactor as DF
    from pgmpy_amd.models import DiscreteMarkovNetwork

    g = DiscreteMarkovNetwork([("a", "b"), ("b", "c")])
    assert sorted(g.nodes()) == ["a", "b", "c"]
    with pytest.raises(ValueError):
        g.add_edge("a", "a")
    with pytest.raises(ValueError):
        g.add_edges_from([("a", "a")])
    assert sorted(g.markov_blanket("b")) == ["a", "c"]
    g = DiscreteMarkovNetwork([("a", "b"), ("b", "c"), ("c", "d"), ("d", "a")])
    assert dict(g.get_cardinality()) == {}
    p1 = DF(["a", "b"], [1, 2], np.random.rand(2))
    g.add_factors(p1)
    assert dict(g.get_cardinality()) == {"a": 1, "b": 2}
    with pytest.raises(ValueError):  # factors missing for c, d
        g.check_model()
    g.remove_factors(p1)
    p1 = DF(["a", "b"], [1, 2], np.random.rand(2))
    p2 = DF(["c", "b"], [3, 2], np.random.rand(6))
    p3 = DF(["c", "d"], [3, 4], np.random.rand(12))
    p4 = DF(["d", "a"], [4, 1], np.random.rand(4))
    g.add_factors(p1, p2, p3, p4)
    assert g.check_model()
    assert g.get_cardinality("d") == 4
    assert g.states == {"a": [0], "b": [0, 1], "c": [0, 1, 2], "d": [0, 1, 2, 3]}
    assert g.get_factors("a") == [p1, p4]
    g.add_factors(DF(["d", "b"], [4, 2], np.random.rand(8)))  # d-b is not an edge
    with pytest.raises(ValueError, match="inconsistent"):
        g.check_model()
    g2 = DiscreteMarkovNetwork([("a", "b"), ("b", "c")])
    g2.add_factors(DF(["a", "b"], [1, 2], np.random.rand(2)), DF(["b", "c"], [3, 3], np.random.rand(9)))
    with pytest.raises(ValueError, match="Cardinality"):
        g2.check_model()
    with pytest.raises(ValueError):
        g2.add_factors(DF(["a", "x"], [2, 2], np.random.rand(4)))
    with pytest.raises(ValueError):
        g2.get_factors("zz")
    # copy: structure and factors are independent of the original (test_DiscreteMarkovNetwork.py:593-673)
    g3 = DiscreteMarkovNetwork([("a", "b")])
    c = g3.copy()
    g3.add_edges_from([("c", "b")])
    assert len(c.nodes()) == 2 and c.get_factors() == []
    g3.add_nodes_from(["d"])
    assert list(g3.copy().neighbors("d")) == []


def test_markov_conversions_structure():
    from pgmpy_amd.factors.discrete import DiscreteFactor as DF
    from pgmpy_amd.models import DiscreteMarkovNetwork, FactorGraph

    g = DiscreteMarkovNetwork([("Alice", "Bob"), ("Bob", "Charles")])
    with pytest.raises(ValueError):
        g.to_factor_graph()
    p1, p2 = DF(["Alice", "Bob"], [3, 2], np.random.rand(6)), DF(["Bob", "Charles"], [2, 2], np.random.rand(4))
    g.add_factors(p1, p2)
    fg = g.to_factor_graph()
    assert isinstance(fg, FactorGraph)
    assert sorted(map(str, fg.nodes())) == ["Alice", "Bob", "Charles", "phi_Alice_Bob", "phi_Bob_Charles"]
    assert fg.get_factors() == [p1, p2]
    cyc = _model(G["cycle4"])
    bm = cyc.to_bayesian_model()
    import networkx as nx

    assert sorted(bm.nodes()) == ["a", "b", "c", "d"]
    assert nx.is_chordal(bm.to_undirected())
    fg = FactorGraph()
    fg.add_nodes_from(["a", "b", "c", "d"])
    fg.add_factors(*cyc.factors)
    fg.add_nodes_from(cyc.factors)
    fg.add_edges_from([(v, f) for f in cyc.factors for v in f.variables])
    assert sorted(sorted(e) for e in fg.to_markov_model().edges()) == G["factor_graph_to_markov_edges"]


def test_alarm_to_markov_model_structure():
    from pgmpy_amd.utils import get_example_model

    am = get_example_model("alarm").to_markov_model()
    assert sorted(sorted(e) for e in am.edges()) == G["alarm_markov"]["edges"]
    assert am.check_model() and len(am.factors) == 37


def test_cluster_graph_and_junction_tree_containers():
    """ClusterGraph.py:63-365, JunctionTree.py:55-114."""
    from pgmpy_amd.factors.discrete import DiscreteFactor as DF
    from pgmpy_amd.models import ClusterGraph, JunctionTree

    cg = ClusterGraph()
    with pytest.raises(TypeError):
        cg.add_node("a")
    cg.add_nodes_from([("a", "b", "c"), ("a", "b"), ("a", "c")])
    cg.add_edges_from([(("a", "b", "c"), ("a", "b")), (("a", "b", "c"), ("a", "c"))])
    cg.add_edge(("a", "b"), ("a", "c"))  # cluster graphs may have cycles
    with pytest.raises(ValueError, match="sepset"):
        cg.add_edge(("a", "b"), ("c", "d"))
    p1 = DF(["a", "b", "c"], [2, 2, 2], np.random.rand(8))
    p2 = DF(["a", "b"], [2, 2], np.random.rand(4))
    with pytest.raises(ValueError):
        cg.add_factors(DF(["a", "d"], [2, 2], np.random.rand(4)))
    cg.add_factors(p1, p2)
    with pytest.raises(ValueError, match="cliques or clusters"):
        cg.check_model()
    p3 = DF(["a", "c"], [2, 2], np.random.rand(4))
    cg.add_factors(p3)
    assert cg.check_model()
    assert cg.get_factors(("b", "a")) is p2
    assert set(cg.clique_beliefs) == set(cg.nodes())
    assert dict(cg.get_cardinality()) == {"a": 2, "b": 2, "c": 2}
    cp = cg.copy()
    assert isinstance(cp, ClusterGraph) and len(cp.factors) == 3 and cp.factors[0] is not p1
    jt = JunctionTree([(("a", "b"), ("b", "c")), (("b", "c"), ("c", "d"))])
    with pytest.raises(ValueError, match="cycle"):
        jt.add_edge(("a", "b"), ("c", "d"))
    jt.add_node(("x", "y"))
    jt.add_factors(DF(["a", "b"], [2, 3], range(6)), DF(["b", "c"], [3, 2], range(6)), DF(["c", "d"], [2, 2], range(4)),
                   DF(["x", "y"], [2, 2], range(4)))
    with pytest.raises(ValueError, match="connected"):
        jt.check_model()


# ----------------------------------------------------------------------------- device inference (GPU)
@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_markov_variable_elimination(gpu, name):
    from pgmpy_amd.inference import VariableElimination

    case = G[name]
    ve = VariableElimination(_model(case))
    for q in case["queries"]:
        r = ve.query(q["variables"], q["evidence"], show_progress=False)
        _close(_values(r, q["joint"]["variables"]), q["joint"])
        sep = ve.query(q["variables"], q["evidence"], joint=False, show_progress=False)
        for v, fj in q["separate"].items():
            _close(sep[v].values, fj)
        r2 = ve.query(q["variables"], q["evidence"], elimination_order=q["order"], show_progress=False)
        _close(_values(r2, q["joint_order"]["variables"]), q["joint_order"])
    for m in case["maps"]:
        got = ve.map_query(m["variables"], m["evidence"], show_progress=False)
        assert {k: str(v) for k, v in got.items()} == m["result"]
    for m in case["max_marginals"]:
        got = ve.max_marginal(m["variables"], m["evidence"], show_progress=False)
        assert got == pytest.approx(m["result"], rel=1e-12)
    assert _model(case).get_partition_function() == pytest.approx(case["partition_function"], rel=1e-12)


@pytest.mark.gpu
def test_markov_samiam_values_and_duplicates(gpu):
    """test_ExactInference.py:639-830 asserted through DiscreteFactor.__eq__, as the reference does."""
    from pgmpy_amd.factors.discrete import DiscreteFactor
    from pgmpy_amd.inference import VariableElimination

    ve = VariableElimination(_model(G["markov6"]))
    for _ in range(2):  # querying twice leaves the model unchanged (test_query_multiple_times)
        assert ve.query(["J"], show_progress=False) == DiscreteFactor(["J"], [2], np.array([0.416, 0.584]))
        assert ve.query(["Q", "J"], show_progress=False) == DiscreteFactor(
            ["Q", "J"], [2, 2], np.array([[0.3744, 0.1168], [0.0416, 0.4672]]))
        assert ve.query(["J"], {"A": 0, "R": 1}, show_progress=False) == DiscreteFactor(["J"], [2], [0.072, 0.048])
        assert ve.query(["J", "Q"], {"A": 0, "R": 0, "G": 0, "L": 1}, show_progress=False) == DiscreteFactor(
            ["J", "Q"], [2, 2], np.array([[0.003888, 0.000432], [0.000192, 0.000768]]))
    for vs in ([], ["G"], ["G", "R"], ["G", "R", "A"]):
        np.testing.assert_almost_equal(ve.max_marginal(vs or None), 0.1659, decimal=4)
    assert ve.map_query(show_progress=False) == {"A": 1, "R": 1, "J": 1, "Q": 1, "G": 0, "L": 0}
    assert ve.map_query(["A", "R", "L"], {"J": 0, "Q": 1, "G": 0}, show_progress=False) == {"A": 1, "R": 0, "L": 0}
    ig = ve.induced_graph(["G", "Q", "A", "J", "L", "R"])
    assert sorted(sorted(e) for e in ig.edges()) == G["markov6"]["induced_graph"]
    assert ve.induced_width(["G", "Q", "A", "J", "L", "R"]) == G["markov6"]["induced_width"]
    d = G["duplicated"]
    from pgmpy_amd.models import DiscreteMarkovNetwork

    dup = DiscreteMarkovNetwork([("A", "B"), ("A", "C")])
    dup.add_factors(*[DiscreteFactor(f["variables"], f["cardinality"], fac_values(f)) for f in d["factors"]])
    assert VariableElimination(dup).query(["A"], show_progress=False) == DiscreteFactor(["A"], [2], np.array([4, 4]))


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_markov_junction_tree_and_belief_propagation(gpu, name):
    from pgmpy_amd.inference import BeliefPropagation

    case = G[name]
    mm = _model(case)
    jt = mm.to_junction_tree()
    if name in TIE_FREE:
        assert sorted(sorted(c) for c in jt.nodes()) == case["jt_cliques"]
        assert len(jt.edges()) == len(case["jt_edges"])
    assert jt.check_model()
    facs = _ofactors(case)
    # the product of the clique potentials is the product of the network's potentials
    assert jt.get_partition_function() == pytest.approx(case["partition_function"], rel=1e-12)
    for op, key in (("calibrate", "bp_clique_beliefs"), ("max_calibrate", "bp_max_clique_beliefs")):
        bp = BeliefPropagation(mm)
        getattr(bp, op)()
        got = {tuple(sorted(c)): f for c, f in bp.get_clique_beliefs().items()}
        compared = 0
        for c, fj in case[key]:  # the reference's cliques (all of them when the structure has no ties)
            if tuple(c) in got:
                _close(_values(got[tuple(c)], c), fj)
                compared += 1
            elif op == "calibrate":
                # a clique of the reference's tree that a tie gave a different shape here: its calibrated
                # belief is the unnormalised marginal Z P(c), which this build's BP answers as a query
                r = BeliefPropagation(mm).query(list(fj["variables"]), joint=True, show_progress=False)
                z = jt.get_partition_function()
                np.testing.assert_allclose(_values(r, fj["variables"]) * z, fac_values(fj), rtol=1e-9, atol=1e-12)
                compared += 1
        # nothing vacuous: every case compares cliques (in the tie cases at least one clique is shared
        # for the max-product beliefs, and every reference clique is checked for the sum-product ones)
        assert compared > 0 and (op == "max_calibrate" or compared == len(case[key]))
        if op == "calibrate":
            # every calibrated clique belief is the unnormalised marginal of the network over the clique
            for c, f in got.items():
                exp = OM.query(facs, list(c), {})
                np.testing.assert_allclose(_values(f, list(c)), exp, rtol=1e-10, atol=1e-12)
            seps = {tuple(sorted(tuple(sorted(x)) for x in k)): f for k, f in bp.get_sepset_beliefs().items()}
            n_sep = 0
            for k, fj in case["bp_sepset_beliefs"]:
                if tuple(tuple(x) for x in k) in seps:
                    _close(_values(seps[tuple(tuple(x) for x in k)], fj["variables"]), fj)
                else:  # a sepset of the reference's tree only: Z P(S) through the build's BP
                    r = BeliefPropagation(mm).query(list(fj["variables"]), joint=True, show_progress=False)
                    np.testing.assert_allclose(_values(r, fj["variables"]) * jt.get_partition_function(),
                                               fac_values(fj), rtol=1e-9, atol=1e-12)
                n_sep += 1
            assert n_sep == len(case["bp_sepset_beliefs"]) > 0
    for q in case["bp_queries"]:
        r = BeliefPropagation(mm).query(q["variables"], q["evidence"], show_progress=False)
        _close(_values(r, q["joint"]["variables"]), q["joint"])
        m = BeliefPropagation(mm).map_query(q["variables"], q["evidence"], show_progress=False)
        assert {k: str(v) for k, v in m.items()} == q["map"]


@pytest.mark.gpu
def test_alarm_as_markov_network(gpu):
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    ve = VariableElimination(get_example_model("alarm").to_markov_model())
    for q in G["alarm_markov"]["queries"]:
        r = ve.query(q["variables"], q["evidence"], show_progress=False)
        _close(_values(r, q["joint"]["variables"]), q["joint"], atol=1e-15)
