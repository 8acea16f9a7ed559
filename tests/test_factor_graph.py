"""FactorGraph + BeliefPropagationWithMessagePassing.

Known-answer values are the reference's own test expectations
(pgmpy/tests/test_inference/test_ExactInference.py:1165-1346, transcribed numbers) on its
4-variable factor graph; the graph structure checks (FactorGraph.py:205-247) run on the host."""
import numpy as np
import pytest


def _graph():
    from pgmpy_amd.factors.discrete import DiscreteFactor
    from pgmpy_amd.models import FactorGraph

    G = FactorGraph()
    G.add_nodes_from(["A", "B", "C", "D"])
    phi1 = DiscreteFactor(["A"], [2], [0.4, 0.6])
    phi2 = DiscreteFactor(["B", "A"], [3, 2], [[0.2, 0.05], [0.3, 0.15], [0.5, 0.8]])
    phi3 = DiscreteFactor(["C", "B"], [2, 3], [[0.4, 0.5, 0.1], [0.6, 0.5, 0.9]])
    phi4 = DiscreteFactor(["D", "B"], [3, 3], [[0.1, 0.1, 0.2], [0.3, 0.2, 0.1], [0.6, 0.7, 0.7]])
    G.add_factors(phi1, phi2, phi3, phi4)
    G.add_edges_from([(phi1, "A"), ("A", phi2), (phi2, "B"), ("B", phi3), (phi3, "C"), ("B", phi4), (phi4, "D")])
    return G, (phi1, phi2, phi3, phi4)


def test_factor_graph_structure_host():
    from pgmpy_amd.factors.discrete import DiscreteFactor
    from pgmpy_amd.models import FactorGraph

    G, (phi1, phi2, phi3, phi4) = _graph()
    assert G.check_model()
    assert sorted(G.get_variable_nodes()) == ["A", "B", "C", "D"]
    assert len(G.get_factor_nodes()) == 4
    assert G.get_factors(phi2) == phi2
    assert G.get_cardinality("B") == 3
    assert dict(G.get_cardinality()) == {"A": 2, "B": 3, "C": 2, "D": 3}
    np.testing.assert_array_equal(G.get_point_mass_message("B", 2), [0, 0, 1])
    np.testing.assert_allclose(G.get_uniform_message("D"), [1 / 3] * 3)
    with pytest.raises(ValueError):
        G.add_edge("A", "A")
    bad = FactorGraph()
    bad.add_nodes_from(["x", "y"])
    bad.add_edge("x", "y")  # variable-variable edge
    bad.add_factors(DiscreteFactor(["x", "y"], [2, 2], np.ones(4)))
    with pytest.raises(ValueError):
        bad.check_model()
    H = G.copy()
    assert H.check_model() and len(H.factors) == 4


@pytest.mark.gpu
def test_message_passing_known_answers(gpu):
    from pgmpy_amd.factors.discrete import TabularCPD
    from pgmpy_amd.inference import BeliefPropagationWithMessagePassing

    G, _ = _graph()
    bp = BeliefPropagationWithMessagePassing(G)
    res = bp.query(["C"])
    np.testing.assert_allclose(res["C"].values, [0.217, 0.783], rtol=1e-9)
    res = bp.query(["A", "B", "C", "D"])
    np.testing.assert_allclose(res["A"].values, [0.4, 0.6], rtol=1e-9)
    np.testing.assert_allclose(res["B"].values, [0.11, 0.21, 0.68], rtol=1e-9)
    np.testing.assert_allclose(res["C"].values, [0.217, 0.783], rtol=1e-9)
    np.testing.assert_allclose(res["D"].values, [0.168, 0.143, 0.689], rtol=1e-9)
    res = bp.query(["B", "C"], {"A": 1, "D": 0})
    np.testing.assert_allclose(res["B"].values, [0.02777778, 0.08333333, 0.88888889], atol=1e-8)
    np.testing.assert_allclose(res["C"].values, [0.14166667, 0.85833333], atol=1e-8)
    res = bp.query(["B"], virtual_evidence=[TabularCPD("A", 2, [[0.1], [0.9]])])
    np.testing.assert_allclose(res["B"].values, [0.06034483, 0.16034483, 0.77931034], atol=1e-8)
    ve = [TabularCPD("A", 2, [[0.027], [0.972]]), TabularCPD("B", 3, [[0.3], [0.6], [0.1]])]
    res = bp.query(["B", "C"], evidence={"D": 0}, virtual_evidence=ve)
    np.testing.assert_allclose(res["B"].values, [0.05938567, 0.3440273, 0.59658703], atol=1e-8)
    np.testing.assert_allclose(res["C"].values, [0.25542662, 0.74457338], atol=1e-8)
    res1 = bp.query(["B"], virtual_evidence=[TabularCPD("A", 2, [[0.1], [0.9]]), TabularCPD("A", 2, [[0.3], [0.7]])])
    np.testing.assert_allclose(res1["B"].values, [0.05461538, 0.15461538, 0.79076923], atol=1e-8)
    with pytest.raises(ValueError):
        bp.query(["B"], evidence={"A": 1}, virtual_evidence={"A": [np.array([0.1, 0.9])]})


@pytest.mark.gpu
def test_message_passing_messages(gpu):
    from pgmpy_amd.inference import BeliefPropagationWithMessagePassing

    G, _ = _graph()
    bp = BeliefPropagationWithMessagePassing(G)
    res, messages = bp.query(["B"], get_messages=True)
    np.testing.assert_allclose(res["B"].values, [0.11, 0.21, 0.68], rtol=1e-9)
    np.testing.assert_allclose(messages["['A'] -> A"], [0.4, 0.6])
    np.testing.assert_allclose(messages["A -> ['B', 'A']"], [0.4, 0.6])
    np.testing.assert_allclose(messages["['B', 'A'] -> B"], [0.11, 0.21, 0.68])
    np.testing.assert_allclose(messages["C -> ['C', 'B']"], [0.5, 0.5])
    np.testing.assert_allclose(messages["['C', 'B'] -> B"], [1 / 3] * 3)
    np.testing.assert_allclose(messages["D -> ['D', 'B']"], [1 / 3] * 3)
    np.testing.assert_allclose(messages["['D', 'B'] -> B"], [1 / 3] * 3)
    res, messages = bp.query(["C", "B"], get_messages=True)
    np.testing.assert_allclose(messages["['C', 'B'] -> C"], [0.217, 0.783])
    res, messages = bp.query(["A"], get_messages=True)
    res2, messages2 = bp.query(["A"], get_messages=True, precomp_messages={"['B', 'A'] -> A": np.array([0.5, 0.5])})
    np.testing.assert_allclose(res2["A"].values, res["A"].values)
    np.testing.assert_allclose(messages2["['B', 'A'] -> A"], messages["['B', 'A'] -> A"])
    assert G.get_partition_function() == pytest.approx(1.0)
