"""The launch-hazard check (pgmpy_amd/hazard.py, Program.check_hazards) on the programs the engine
really builds: the C4 pathfinder batched calibration (1,000 and 4,000 rows, sum and max), the C2 munin
query program and alarm's query programs.  Every launch's byte ranges
are recomputed from its own descriptor; the check fails on any range outside the buffers a launch
declares or any overlapping pair (one writing) the schedule does not order.  Programs are built on
the device (their buffers are real allocations); the check itself launches nothing."""
import random

import pytest

from tests.goldens import load_json

pytestmark = pytest.mark.gpu


def _jt(model, meta):
    from pgmpy_amd.inference.EliminationOrder import build_junction_tree

    bags = [tuple(b) for b in meta["bags"]]
    edges = [(tuple(a), tuple(b)) for a, b in meta["edges"]]
    return build_junction_tree(model, bags, edges)


@pytest.mark.parametrize("rows,op", [(1000, "marginalize"), (4000, "marginalize"), (1000, "maximize")])
def test_c4_schedule_has_no_unordered_overlap(gpu, rows, op):
    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.utils import get_example_model

    m = get_example_model("pathfinder")
    bjt = BatchedJunctionTree(_jt(m, load_json("pathfinder_bp.json")))
    leaves = sorted(n for n in m.nodes() if m.out_degree(n) == 0)
    sch = bjt.schedule(rows, leaves, op, marginals=True, graph=False)
    prog = sch.prog
    assert prog._levels and len(prog._recs) > 100
    assert all(r.foot for r in prog._recs), [r.note for r in prog._recs if not r.foot][:3]
    assert prog.check_hazards() == []


def test_c2_and_alarm_programs_have_no_unordered_overlap(gpu):
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    leaves = sorted(n for n in m.nodes() if m.out_degree(n) == 0)
    roots = sorted(n for n in m.nodes() if m.in_degree(n) == 0)
    rng = random.Random(100000)
    E = rng.sample(leaves, 100)
    q = [rng.choice(roots)]
    codes, nodes = forward_sample_codes(m, 1, seed=0)
    ev = {v: m.states[v][codes[nodes.index(v), 0]] for v in E}
    ve = VariableElimination(m)
    ve.query(q, ev, show_progress=False)
    progs = [p for r in ve._compiled.values() for p, *_ in r.plan.__dict__.get("_progs", {}).values()]
    assert progs, "the C2 query compiled no steps program"
    a = get_example_model("alarm")
    vea = VariableElimination(a)
    nodes_a = sorted(a.nodes())
    rng = random.Random(1)
    ca, na = forward_sample_codes(a, 20, seed=1)
    for r in range(20):
        pick = rng.sample(nodes_a, 8)
        vea.query(pick[:3], {v: a.states[v][ca[na.index(v), r]] for v in pick[3:]}, show_progress=False)
    progs += [p for r in vea._compiled.values() for p, *_ in r.plan.__dict__.get("_progs", {}).values()]
    for p in progs:
        assert not p._levels
        assert p._plain_recs and all(r.foot for r in p._plain_recs)
        assert p.check_hazards() == []
