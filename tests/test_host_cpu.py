"""Host-side logic that needs no GPU: the C-ABI library, BIF reader, pruning, planners, encoding.

The library test loads libpgmhip.so and checks it exports every entry point
declared in include/pgmhip.h (no compute call: no device here).
"""
import os
import re

import numpy as np
import pandas as pd
import pytest

from oracle import ve as OVE
from oracle.network import load_network

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    from pgmpy_amd import _native as N
    from pgmpy_amd.build import build

    build(verbose=False)
    lib = N.load_library()
    header = open(os.path.join(ROOT, "include", "pgmhip.h")).read()
    declared = set(re.findall(r"\bint\s+(pgm_[a-z0-9_]+)\s*\(", header))
    assert declared, "no declarations parsed"
    assert declared == set(N.EXPORTED), declared ^ set(N.EXPORTED)
    for name in declared:
        assert hasattr(lib, name)
    assert lib.pgm_version() == 23


def test_struct_layouts_match_header():
    """ctypes mirrors of the descriptors have the C sizes (pgmhip.h)."""
    import ctypes

    from pgmpy_amd import _native as N

    assert ctypes.sizeof(N.ContractDesc) == 16 + 7 * 8 * N.PGM_MAX_DIMS
    assert ctypes.sizeof(N.ContractNDesc) == 16 + (3 + 2 * N.PRODN_MAX_OPS) * 8 * N.PGM_MAX_DIMS
    assert ctypes.sizeof(N.GatherDesc) == 16 + 16 + 6 * 8 * N.PGM_MAX_DIMS
    assert ctypes.sizeof(N.RowsPlan) == 4 * (8 + 3 * N.ROWS_MAX_LOOP + 5 * N.ROWS_MAX_COMP
                                             + N.ROWS_MAX_FAC * (3 + N.ROWS_MAX_LOOP) + 3 * N.ROWS_MAX_EV)


def test_argument_checks_before_any_device_call():
    """Entry points of r03 reject bad arguments on the host, before any HIP call (no device here):
    pgm_rows_shard_run (no handles, a null handle, a mode it does not take, no output),
    pgm_batch_set_mode (an unknown mode) and pgm_batch_blocks (a null handle)."""
    import ctypes

    from pgmpy_amd import _native as N

    lib = N.load_library()
    h = (ctypes.c_void_p * 1)(None)
    codes = np.zeros((1, 4), dtype=np.uint8)
    marg = np.zeros((2, 4))
    args = (codes.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(4), ctypes.c_int64(1), ctypes.c_int64(4),
            marg.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(4), None, None)
    shard = lib.pgm_rows_shard_run
    shard.restype = ctypes.c_int
    assert shard(h, ctypes.c_int32(0), ctypes.c_int32(N.ROWS_MARGINALS), *args) == N.PGM_EINVAL  # no handles
    assert shard(h, ctypes.c_int32(1), ctypes.c_int32(N.ROWS_MARGINALS), *args) == N.PGM_EINVAL  # null handle
    assert shard(h, ctypes.c_int32(1), ctypes.c_int32(N.ROWS_JOINT), *args) == N.PGM_EINVAL  # mode
    assert shard(h, ctypes.c_int32(1), ctypes.c_int32(0), *args) == N.PGM_EINVAL  # no output
    b = ctypes.c_void_p()
    assert lib.pgm_batch_create(ctypes.byref(b)) == 0
    try:
        assert lib.pgm_batch_set_mode(b, ctypes.c_int32(7)) == N.PGM_EINVAL
        assert lib.pgm_batch_set_mode(b, ctypes.c_int32(N.BATCH_ONE_WORKGROUP)) == 0
        n = ctypes.c_int64(-1)
        assert lib.pgm_batch_blocks(b, ctypes.byref(n)) == 0 and n.value == 0
        assert lib.pgm_batch_blocks(None, ctypes.byref(n)) == N.PGM_EINVAL
    finally:
        lib.pgm_batch_destroy(b)


def test_no_compute_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from pgmpy_amd import _native as N
    from pgmpy_amd.factors.discrete import DiscreteFactor

    phi = DiscreteFactor(["a"], [2], [1.0, 2.0])
    with pytest.raises(N.NativeUnavailable):
        phi.normalize(inplace=False)


@pytest.mark.parametrize("net", ["alarm", "munin", "pathfinder"])
def test_bif_reader_matches_reference_export(net):
    """pgmpy_amd.readwrite.BIFReader == the reference BIFReader's CPTs (pinned by the fixture)."""
    from pgmpy_amd.utils import get_example_model

    m = get_example_model(net)
    o = load_network(net)
    assert sorted(m.nodes()) == o.nodes
    for v in o.nodes:
        cpd = m.get_cpds(v)
        assert list(cpd.variables[1:]) == list(o.parents[v])
        assert [str(s) for s in cpd.state_names[v]] == o.states[v]
        np.testing.assert_array_equal(np.asarray(cpd._host).reshape(o.cpts[v].shape), o.cpts[v])


@pytest.mark.parametrize("net,n_ev", [("alarm", 5), ("alarm", 20), ("munin", 40), ("munin", 900)])
def test_pruning_matches_oracle(net, n_ev):
    """Integer Bayes-ball pruning (pgmpy_amd.inference.dsep) against the oracle's restatement of
    inference/base.py:154-212 + DAG.py:864-950."""
    from pgmpy_amd.inference.base import prune_structure
    from pgmpy_amd.utils import get_example_model

    m = get_example_model(net)
    o = load_network(net)
    rng = np.random.default_rng(0)
    nodes = sorted(m.nodes())
    for _ in range(12 if net == "alarm" else 4):
        picks = list(rng.choice(nodes, size=2 + n_ev, replace=False))
        q, e = picks[:2], picks[2:]
        kept, ev = prune_structure(m, q, e)
        keep_o, _ = OVE.prune(o, q, e)
        assert set(kept) == keep_o
        assert kept == [v for v in m.nodes() if v in keep_o]  # model order
        if net == "alarm":
            at = m.active_trail_nodes(q, observed=e)
            for v in q:
                assert at[v] == OVE.active_trail_nodes(o, v, e)


def test_active_trail_nodes_api():
    """active_trail_nodes argument forms and latents (DAG.py:864-950)."""
    from pgmpy_amd.models import DiscreteBayesianNetwork

    g = DiscreteBayesianNetwork([("D", "G"), ("I", "G"), ("G", "L"), ("I", "S")])
    assert g.active_trail_nodes("D") == {"D": {"D", "G", "L"}}
    assert g.active_trail_nodes("D", observed="G") == {"D": {"D", "I", "S"}}
    assert g.active_trail_nodes(["D", "I"], observed=["L"])["D"] == {"D", "I", "S", "G"}
    g.latents = {"S"}
    assert g.active_trail_nodes("I")["I"] == {"I", "G", "L", "D"} - {"D"}
    assert "S" in g.active_trail_nodes("I", include_latents=True)["I"]
    g.add_edge("L", "X")  # structural edits are seen (the int index is rebuilt per epoch)
    assert "X" in g.active_trail_nodes("D")["D"]


def test_state_name_policy():
    """StateNameMixin semantics (state_name.py:8-145): maps, lookup errors, merge policy."""
    from pgmpy_amd.factors.discrete import DiscreteFactor

    a = DiscreteFactor(["x", "y"], [2, 2], np.ones(4), state_names={"x": ["lo", "hi"], "y": [0, 1]})
    assert a.get_state_no("x", "hi") == 1 and a.get_state_names("x", 0) == "lo"
    with pytest.raises(KeyError, match="state: mid is an unknown for variable: x"):
        a.get_state_no("x", "mid")
    b = DiscreteFactor(["x"], [2], np.ones(2))  # numeric names: the textual ones win either way
    for first, second in ((a, b), (b, a)):
        f = first.copy()
        f.add_state_names(second)
        assert f.state_names["x"] == ["lo", "hi"] and f.name_to_no["x"]["hi"] == 1
    c = DiscreteFactor(["x"], [2], np.ones(2), state_names={"x": ["on", "off"]})
    with pytest.raises(ValueError, match="State name conflict detected for variable 'x'"):
        a.copy().add_state_names(c)
    with pytest.raises(ValueError, match="Repeated statenames for variable: x"):
        DiscreteFactor(["x"], [2], np.ones(2), state_names={"x": ["a", "a"]})
    with pytest.raises(ValueError, match="The state names must be for the form"):
        DiscreteFactor(["x"], [2], np.ones(2), state_names={"x": "ab"})
    d = a.copy()
    d.del_state_names(["y"])
    assert "y" not in d.state_names and "y" not in d.name_to_no and "y" not in d.no_to_name
    assert list(a.state_table("x").code_lut(["hi", "zz", "lo", ["unhashable"]])) == [1, -1, 0, -1]


def test_value_token_sees_late_host_edits():
    """A values array read now and edited later changes the CPD's value token, which compiled
    plans compare (the device copy must not go stale)."""
    from pgmpy_amd.factors.discrete import TabularCPD

    cpd = TabularCPD("a", 2, [[0.3], [0.7]])
    t0 = cpd._value_token()
    v = cpd.values
    t1 = cpd._value_token()
    assert cpd._value_token() == t1  # reading alone is not a change
    v[0] = 0.4
    assert cpd._value_token() not in (t0, t1)
    t2 = cpd._value_token()
    cpd.values = np.array([0.5, 0.5])
    assert cpd._value_token() != t2


def test_greedy_planner_contract_semantics():
    from pgmpy_amd.inference.contraction import greedy_path, plan_stats

    labels = [["a", "b"], ["b", "c"], ["c", "d"], ["x"]]
    dims = {"a": 2, "b": 3, "c": 4, "d": 5, "x": 6}
    steps, final = greedy_path(labels, ["a", "d"], dims)
    # x is private and not in the output: summed first
    assert steps[0][0] == "reduce" and steps[0][2] == []
    assert final is not None
    st = plan_stats(labels, ["a", "d"], dims)
    assert st["steps"] == len(steps)


def test_encode_and_group_patterns():
    from pgmpy_amd.inference.batch import encode_frame, group_patterns
    from pgmpy_amd.utils import get_example_model

    m = get_example_model("asia")
    df = pd.DataFrame({"asia": ["yes", "no", None, "no"], "smoke": ["no", "yes", "yes", None]})
    codes = encode_frame(m, df)
    st_asia = list(m.states["asia"])
    assert codes[0, 0] == st_asia.index("yes") and codes[0, 2] == 255 and codes[1, 3] == 255
    groups = group_patterns(codes)
    assert sorted(len(r) for _, r in groups) == [1, 1, 2]
    with pytest.raises(KeyError):
        encode_frame(m, pd.DataFrame({"asia": ["maybe"]}))


def test_encode_frame_categorical_numeric_and_nan():
    """Evidence ingestion fast paths (f-4): categorical columns, NaN in either form, numeric cells
    matching string state names through str() (DiscreteFactor.py:589-597), unknown states."""
    from pgmpy_amd.inference.batch import encode_frame
    from pgmpy_amd.utils import get_example_model

    m = get_example_model("asia")
    st = list(m.states["asia"])
    obj = pd.DataFrame({"asia": ["no", "yes", np.nan, "no", None]})
    cat = obj.astype({"asia": pd.CategoricalDtype(categories=["yes", "no", "unused"])})
    want = [st.index("no"), st.index("yes"), 255, st.index("no"), 255]
    assert list(encode_frame(m, obj)[0]) == want
    assert list(encode_frame(m, cat)[0]) == want
    with pytest.raises(KeyError):
        encode_frame(m, pd.DataFrame({"asia": pd.Categorical(["yes", "maybe"])}))

    from pgmpy_amd.factors.discrete import TabularCPD
    from pgmpy_amd.models import DiscreteBayesianNetwork

    bn = DiscreteBayesianNetwork([("a", "b")])
    bn.add_cpds(TabularCPD("a", 2, [[0.5], [0.5]], state_names={"a": ["0", "1"]}),
                TabularCPD("b", 2, [[0.3, 0.6], [0.7, 0.4]], evidence=["a"], evidence_card=[2],
                           state_names={"b": [0, 1], "a": ["0", "1"]}))
    codes = encode_frame(bn, pd.DataFrame({"a": [1, 0, 1], "b": ["1", "0", 1]}))
    assert codes.tolist() == [[1, 0, 1], [1, 0, 1]]

    # predict(stochastic=True) groups by state codes only where raw value <-> state is one to one
    from pgmpy_amd.inference.batch import _raw_values_ambiguous

    assert not _raw_values_ambiguous(bn, pd.DataFrame({"a": ["1", "0", None]}), ["a"])
    assert not _raw_values_ambiguous(bn, pd.DataFrame({"a": [1, 0, 1]}), ["a"])  # one int dtype
    assert _raw_values_ambiguous(bn, pd.DataFrame({"a": [1, "1", "0"]}), ["a"])  # 1 and "1" merge
    assert not _raw_values_ambiguous(bn, pd.DataFrame({"a": pd.Categorical(["1", "0"])}), ["a"])
    assert _raw_values_ambiguous(bn, pd.DataFrame({"a": pd.Categorical([1, "1"])}), ["a"])


def test_columnar_ingestion_matches_host_encoder():
    """ingest_columnar (categorical frames: zero-copy codes, NaN patterns from the NaN-holding
    columns only, per-column LUTs) gives the host encoder's codes and patterns: shuffled category
    orders, unused and str()-matched categories, NaN in several columns; a cell holding a category
    that is not a state raises the reference's KeyError; other dtypes fall back (None)."""
    from pgmpy_amd.inference.batch import encode_frame, group_patterns, ingest_columnar
    from pgmpy_amd.utils import get_example_model

    m = get_example_model("alarm")
    rng = np.random.default_rng(4)
    cols = sorted(m.nodes())[:12]
    n = 1003  # not a multiple of 8: the NaN scan's tail
    data = {}
    for j, c in enumerate(cols):
        st = [str(s) for s in m.states[c]]
        cats = list(rng.permutation(st)) + (["unused"] if j % 3 == 0 else [])
        codes = rng.integers(0, len(st), n)
        vals = np.array([st[k] for k in codes], dtype=object)
        if j in (2, 5, 9):
            vals[rng.random(n) < 0.05] = None
        data[c] = pd.Categorical(vals, categories=cats)
    df = pd.DataFrame(data)
    ev = ingest_columnar(m, df, cols)
    want = encode_frame(m, df, cols)
    rows = np.arange(n)
    assert np.array_equal(ev.host_codes_for(list(range(len(cols))), rows), want)
    sub = rows[::7]
    assert np.array_equal(ev.host_codes_for([3, 9, 0], sub), want[[3, 9, 0]][:, sub])
    exp = {tuple(np.nonzero(~mk)[0]): set(r.tolist()) for mk, r in group_patterns(want)}
    got = {tuple(np.nonzero(~mk)[0]): set(r.tolist()) for mk, r in ev.groups}
    assert got == exp and len(got) > 3
    bad = df.copy()
    bad[cols[0]] = pd.Categorical([str(m.states[cols[0]][0])] * (n - 1) + ["unused"],
                                  categories=[str(s) for s in m.states[cols[0]]] + ["unused"])
    with pytest.raises(KeyError):
        ingest_columnar(m, bad, cols)
    assert ingest_columnar(m, df.astype({cols[1]: object}), cols) is None
    # r05: the NaN scan left pending (the direct path runs meanwhile), then run on a worker thread and
    # joined, gives the same groups
    dev = ingest_columnar(m, df, cols, defer_scan=True)
    assert dev.groups is None
    dev.start_scan()
    dev.finish_scan()
    assert {tuple(np.nonzero(~mk)[0]): set(r.tolist()) for mk, r in dev.groups} == exp
    # r05: frame-schema cache — a frame whose every category is a state name is ingested through the stored
    # LUTs the second time (same codes); a model structure edit (epoch) misses
    from pgmpy_amd.inference import batch as B

    clean = pd.DataFrame({c: pd.Categorical.from_codes(rng.integers(0, len(m.states[c]), n).astype(np.int8),
                                                       categories=[str(s) for s in m.states[c]]) for c in cols})
    e1 = ingest_columnar(m, clean, cols)
    cats = B._frame_categoricals(clean, cols)
    assert B._schema_fast(m, cols, cats, n) is not None
    e2 = ingest_columnar(m, clean, cols)
    assert all(a is b for a, b in zip(e1.luts, e2.luts))
    assert np.array_equal(e2.host_codes_for(list(range(len(cols))), rows), encode_frame(m, clean, cols))
    assert B._schema_fast(m, cols, B._frame_categoricals(df, cols), n) is None  # "unused" categories: not stored
    m._bump()
    assert B._schema_fast(m, cols, cats, n) is None


def test_specialised_row_kernel_source_compiles_for_gfx950():
    """pgm_rows_plan_source (host-only) emits the C3 template's specialised kernel: every evidence
    column loaded once, one store per marginal entry, and it compiles for gfx950 with hipcc."""
    import random
    import shutil
    import subprocess
    import tempfile

    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    obs = sorted(v for v in m.nodes() if v not in missing)
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    assert plan.kernel_name() == "pgm_rows_jit"
    src = plan.specialised_source()
    one_row = src[:src.index("pgm_rows_jit2(")]
    assert one_row.count("M[") == plan.n_acc == 17
    assert one_row.count("cr[") == 7  # the template's 7 evidence columns
    # the dispatch floors: same loads and stores, no CPT math (one-row and two-row grids)
    floor = src[src.index("pgm_rows_floor("):src.index("pgm_rows_floor2(")]
    assert floor.count("M[") == 17 and floor.count("cr[") == 7 and "S[" not in floor
    floor2 = src[src.index("pgm_rows_floor2("):src.index("struct pgm_ring_slot")]
    assert floor2.count("(cr + ") == 7 and floor2.count("PGM_WT16(rsM") == 17 and "S[" not in floor2
    # the resident ring kernel: the two-row body once per 128-row work item, the host counter polled
    # with a system-scope acquire, a timeout every waiting wave checks
    ring = src[src.index("pgm_rows_ring("):]
    assert ring.count("(cr + ") == 7 and ring.count("PGM_WT16(rsM") == 17
    assert "__HIP_MEMORY_SCOPE_SYSTEM" in ring and ring.count("> timeout") == 3 and "if (r >= n) break;" in ring
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "k.hip")
        with open(path, "w") as f:
            f.write(src)
        r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-x", "hip", "-include", "hip/hip_runtime.h",
                            "--cuda-device-only", "-c", path, "-o", os.path.join(d, "k.o")],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_program_dependency_levels():
    """Levelled Program (pgmpy_amd/program.py): RAW, WAR and WAW hazards order steps into levels;
    independent steps share a level; views of one buffer conflict.  No launches (host only)."""
    import torch

    from pgmpy_amd.program import Program

    a, b, c, d = (torch.zeros(8) for _ in range(4))
    prog = Program(levels=True)
    ran = []

    def step(name):
        return lambda s: ran.append(name)

    prog._emit(step("w_a"), "w_a", [d], [a])            # L0
    prog._emit(step("w_b"), "w_b", [d], [b])            # L0 (independent)
    prog._emit(step("r_ab_w_c"), "r_ab_w_c", [a, b], [c])  # L1 (RAW on a, b)
    prog._emit(step("w_d"), "w_d", [], [d])             # L1 (WAR on d, read at L0)
    prog._emit(step("inplace_c"), "inplace_c", [c, a[2:]], [c])  # L2 (RAW/WAW on c)
    prog._emit(step("w_a_view"), "w_a_view", [], [a[:4]])  # L3 (WAR: a read at L2 through a view)
    assert prog.n_levels == 4
    assert [r.level for r in prog._recs] == [0, 0, 1, 1, 2, 3]
    for f in prog._steps:
        f(None)
    assert ran == ["w_a", "w_b", "r_ab_w_c", "w_d", "inplace_c", "w_a_view"]


def test_program_hazard_check_catches_undeclared_and_unordered_access():
    """Program.check_hazards (pgmpy_amd/hazard.py): byte ranges recomputed from each launch's own
    descriptor must lie in buffers the launch declares, and overlapping launches (one writing) must
    be in different dependency levels.  Host only: CPU tensors stand in for device buffers, the
    launches are never run."""
    import ctypes

    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd import hazard as H
    from pgmpy_amd.program import Program

    a, b, c, scratch = (torch.zeros(16, dtype=torch.float64) for _ in range(4))

    def whole(t, mode):
        return H.view_foot(t, mode)

    def build(declare_b_write=True, stray=False):
        prog = Program(levels=True)
        prog._keep.extend([a, b, c, scratch])
        nop = lambda s: None  # noqa: E731
        prog._emit(nop, "a -> b", [a], [b] if declare_b_write else [],
                   foot=whole(a, H.READ) + whole(b, H.WRITE))
        prog._emit(nop, "b -> c", [b], [c], foot=whole(b, H.READ) + whole(c, H.WRITE))
        prog._emit(nop, "c[0:8] -> a[8:]", [c], [a], foot=whole(c[:8], H.READ) + whole(a[8:], H.WRITE))
        if stray:  # a launch that touches bytes outside every buffer the program holds
            prog._emit(nop, "stray", [], [], foot=[(8, 16, H.WRITE)])
        return prog

    good = build()
    assert good.check_hazards() == []
    assert [r.level for r in good._recs] == [0, 1, 2]
    # the first launch writes b without declaring it: the reader of b lands in the same level
    bad = build(declare_b_write=False).check_hazards()
    assert any("does not declare written" in m for m in bad), bad
    assert any("without an ordering" in m for m in bad), bad
    assert any("no buffer the program holds" in m for m in build(stray=True).check_hazards())

    # descriptor footprints: a contraction's operand spans follow its strides (a transposed view of
    # a [4, 4] buffer reads all 16 entries; its output row 1 is entries 4..7)
    d = N.ContractDesc()
    d.n_keep, d.n_red = 1, 1
    d.keep_card[0], d.red_card[0] = 4, 4
    d.keep_sa[0], d.red_sa[0] = 1, 4  # A^T
    d.keep_sc[0] = 1
    pa, pc = a.data_ptr(), c.data_ptr() + 4 * 8
    foot = H.contract_foot(d, ctypes.c_void_p(pa), None, ctypes.c_void_p(pc))
    assert foot == [(pa, pa + 16 * 8, H.READ), (pc, pc + 4 * 8, H.WRITE)]
    # plain programs: jobs of one batch launch must be independent
    prog = Program()
    prog._keep.extend([a, b])
    prog.begin_batch()
    prog._batch_job("w a", [], [a], whole(a, H.WRITE))
    prog._batch_job("r a", [a], [b], whole(a, H.READ) + whole(b, H.WRITE))
    prog._batch = None
    assert any("without an ordering" in m for m in prog.check_hazards())


def test_predict_output_frame_assembly():
    """predict's result frame (batch._append_columns): the observed columns then the MAP columns, built
    as one block manager over the input's blocks plus one block per new column, equals pd.concat's
    frame (dtypes, order, index) on mixed block layouts (multi-column float block, categoricals, a
    non-default index)."""
    import os

    from pgmpy_amd.inference.batch import _append_columns

    base = pd.DataFrame({"a": pd.Categorical(["x", "y", "x", "y"]), "f1": [1.0, 2, 3, 4], "f2": [0.5, 0, 1, 2],
                         "c": pd.Categorical(["u", "u", "v", "u"])}, index=[5, 3, 9, 1])
    vals = {"p": np.array(["s0", "s1", "s0", "s1"], dtype=object), "q": np.array([np.nan, "t", "t", "r"], dtype=object)}
    got = _append_columns(base, vals, ["p", "q"])
    old = os.environ.get("PGM_API_APPEND")
    os.environ["PGM_API_APPEND"] = "concat"
    try:
        want = _append_columns(base, vals, ["p", "q"])
    finally:
        if old is None:
            os.environ.pop("PGM_API_APPEND")
        else:
            os.environ["PGM_API_APPEND"] = old
    assert got.equals(want) and list(got.columns) == list(want.columns)
    assert list(got.dtypes) == list(want.dtypes) and list(got.index) == [5, 3, 9, 1]
    assert list(base.columns) == ["a", "f1", "f2", "c"]  # the input frame is not modified


def test_query_name_checks_cached_per_model_structure(monkeypatch):
    """VariableElimination.query skips the variable-name checks for a (query, evidence) name pair it
    already checked, keyed on the model's structure epoch (ExactInference.py, C2 host path); the checks
    themselves still raise as the reference does (ExactInference.py:292-300)."""
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.inference import plan as P
    from pgmpy_amd.utils import get_example_model

    class Runner:  # the device replay replaced by a constant: only the host path is under test
        def __init__(self, plan, joint):
            self.plan, self.joint = plan, joint

        def run(self, codes):
            assert len(codes) == len(self.plan.evidence_vars)
            return np.full(self.plan.P if self.joint else self.plan.n_acc, 0.5)

    monkeypatch.setattr(P, "QueryRunner", Runner)
    m = get_example_model("alarm")
    ve = VariableElimination(m)
    ev = {"HR": "LOW", "CVP": "NORMAL"}
    for _ in range(2):
        f = ve.query(["BP"], ev, show_progress=False)
        assert f.variables == ["BP"] and f.state_names["BP"] == m.states["BP"]
    assert len(ve._valid_keys) == 1
    with pytest.raises(ValueError):
        ve.query(["BP"], {**ev, "BP": "LOW"}, show_progress=False)
    with pytest.raises(KeyError):
        ve.query(["BP"], {"HR": "NOPE", "CVP": "NORMAL"}, show_progress=False)
    from pgmpy_amd.factors.discrete import TabularCPD

    m.add_node("extra")  # a structural change: the names are checked again
    m.add_cpds(TabularCPD("extra", 2, [[0.5], [0.5]]))
    ve.query(["BP"], ev, show_progress=False)
    assert len(ve._valid_keys) == 2


def test_host_delivery_rejects_unknown_mode():
    """HostDelivery's ordering knob is one of three named modes (pgmpy_amd/distributed.py); a typo is an
    error, not a silent fallback to another ordering."""
    from pgmpy_amd.distributed import HostDelivery

    assert HostDelivery.MODES == ("lanes", "same", "separate")
    with pytest.raises(ValueError, match="not one of"):
        HostDelivery((4,), None, mode="overlap")


def test_device_lock_readers_writer_semantics():
    """engine.DeviceLock (SURVEY §8(b) threading): shared holds overlap across threads, an exclusive
    hold excludes everyone, holds nest, and two threads that each hold it shared and then ask for it
    exclusively (a capture inside a public call) both get it in turn instead of deadlocking."""
    import threading
    import time

    from pgmpy_amd.engine import DeviceLock

    lk = DeviceLock()
    inside, peak, errors = [0], [0], []
    gate = threading.Barrier(4)

    def reader():
        with lk.shared():
            with lk.shared():  # re-entrant
                gate.wait(timeout=5)  # all four readers inside at once
                inside[0] += 1
                peak[0] = max(peak[0], inside[0])
                time.sleep(0.01)
                inside[0] -= 1

    ts = [threading.Thread(target=reader) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert lk.peak_readers == 4 and peak[0] >= 2

    order = []

    def upgrader(tag):
        try:
            with lk.shared():
                time.sleep(0.02)
                with lk.exclusive():  # gives the shared hold up while waiting
                    order.append((tag, "in"))
                    with lk.shared():  # shared inside exclusive: free
                        pass
                    with lk.exclusive():  # nested exclusive
                        pass
                    time.sleep(0.01)
                    order.append((tag, "out"))
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    ts = [threading.Thread(target=upgrader, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert not any(t.is_alive() for t in ts), "deadlock"
    assert not errors
    # exclusive sections did not interleave
    assert [o[1] for o in order] == ["in", "out", "in", "out"] and order[0][0] == order[1][0]
    # after everything: free for a new exclusive holder at once
    done = threading.Event()
    threading.Thread(target=lambda: (lk.acquire_exclusive(), lk.release_exclusive(), done.set())).start()
    assert done.wait(5)


def test_hip_backend_config_mirrors_pgmpy_config():
    """pgmpy_amd.compat.Config: pgmpy's set_backend validation (global_vars.py:82-122) plus "hip";
    without a device the hip backend fails loudly (no CPU fallback)."""
    from pgmpy_amd import compat
    from pgmpy_amd._native import NativeUnavailable

    cfg = compat.Config()
    assert cfg.get_backend() == "numpy" and cfg.get_dtype() == "float64"
    with pytest.raises(ValueError):
        cfg.set_backend("jax")
    import torch

    if not torch.cuda.is_available():
        with pytest.raises(NativeUnavailable):
            cfg.set_backend("hip")
        assert compat.get_compute_backend() is np  # module config untouched
    cfg.set_backend("numpy")
    assert cfg.get_device() is None


def _pm_desc(N, shapes_labels, out_labels, card, kinds=None):
    """ProductNDesc for C-order operands (numpy element strides), out C-order over out_labels."""
    import numpy as np

    d = N.ProductNDesc()
    d.n_ops, d.n_keep = len(shapes_labels), len(out_labels)
    for i, k in enumerate(kinds or []):
        d.op_kind[i] = int(k)
    out_shape = [card[l] for l in out_labels]
    out_st = [s // 8 for s in np.empty(out_shape).strides]
    for i, l in enumerate(out_labels):
        d.keep_card[i], d.keep_sc[i] = card[l], out_st[i]
        for t, ls in enumerate(shapes_labels):
            st = [s // 8 for s in np.empty([card[x] for x in ls]).strides]
            d.keep_s[t][i] = st[ls.index(l)] if l in ls else 0
    return d


@pytest.mark.parametrize("red,store,ratio,short", [(1, True, False, False), (2, True, True, False),
                                                   (1, False, True, False), (1, False, False, True)])
def test_product_marginal_specialised_source_compiles(tmp_path, red, store, ratio, short):
    """The specialised product+marginal kernel the bind entry point would compile (hipRTC on the
    GPU box) is generated on the host and compiles for gfx950 with hipcc: literal outer decode,
    nested reduced loops, ratio operands, marginal-only form."""
    import ctypes
    import shutil
    import subprocess

    import numpy as np

    from pgmpy_amd import _native as N

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    L = N.load_library()
    R = "__row__"
    card = dict(zip(list("abcdef") + [R], (8, 2, 3, 8, 5, 9, 4000 if short else 2100)))
    cl = list("abcdef") + [R]
    ops = [list("abcdef"), ["a", "c", "f", R]]
    kinds = None
    if ratio:
        ops = [cl, ["a", "d", "f", R], ["a", "d", "f", R]]
        kinds = [N.PRODN_MUL, N.PRODN_RATIO, N.PRODN_DEN]
    d = _pm_desc(N, ops, cl, card, kinds)
    # short: a marginal over one 2-state dim (a separator message from a small operand) — too little
    # work per lane for one row pair, so the generator gives each lane 4 (x0..x3)
    marg = ["a", "c", "d", "e", "f", R] if short else ["a", "d", "e", R]
    m_st = [s // 8 for s in np.empty([card[x] for x in marg]).strides]
    ms = (ctypes.c_int64 * len(cl))(*[m_st[marg.index(l)] if l in marg else 0 for l in cl])
    fake = [0x10000000 * (i + 1) for i in range(len(ops))]  # 16-B aligned, never dereferenced
    ptrs = (ctypes.c_void_p * len(ops))(*fake)
    buf = ctypes.create_string_buffer(1 << 16)
    n = L.pgm_product_n_marginal_source(ctypes.byref(d), ptrs, ctypes.c_void_p(0x70000000) if store else None, ms,
                                        red, ctypes.c_void_p(0x60000000), buf, len(buf))
    assert n > 0, "shape should specialise"
    src = buf.value.decode()
    assert "pgm_pm" in src and ("* pgm_ratio(" in src) == ratio
    assert ("cj[" in src or "nontemporal_store(w" in src or "raw_buffer_store_b128(q_" in src) == store
    assert ("const unsigned x3 = " in src) == short
    f = tmp_path / "pm.hip"
    f.write_text("#include <hip/hip_runtime.h>\n" + src)
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-c", str(f), "-o",
                        str(tmp_path / "pm.o")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]


def test_bench_cpu_baselines_run():
    """bench.py's cpu_baseline legs (numpy oracle, 1 core and the worker pool) run on a small sample
    and report positive rates (the bench line carries them; no GPU involved)."""
    import argparse
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    one, allcore = bench.cpu_baselines_c3(argparse.Namespace(rows=300, cpu_seconds=0.5))
    assert one["value"] > 0 and one["cores"] == 1 and one["kind"] == "port"
    assert allcore["value"] > 0 and allcore["cores"] >= 1


def test_c4_junction_tree_is_the_golden_tree():
    """bench.py's C4 line builds its tree with junction_tree_from_model (min-fill decomposition); the
    pathfinder BP fixture (tests/golden/pathfinder_bp.json) holds the reference's beliefs on a tree the
    generator built the same way. They must be the same tree: bags in the same order (bags[0] is
    the sweep's root) and the same edges."""
    import json

    from pgmpy_amd.inference.EliminationOrder import min_fill_decomposition
    from pgmpy_amd.utils import get_example_model

    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "pathfinder_bp.json")))
    bags, edges = min_fill_decomposition(get_example_model("pathfinder"))
    assert bags == [tuple(b) for b in meta["bags"]]
    assert {frozenset(e) for e in edges} == {frozenset((tuple(a), tuple(b))) for a, b in meta["edges"]}


def test_c4_leaf_findings_shape():
    """The C4 evidence generator: every leaf a column, exactly 4 findings per row, the rest 255, each
    finding the row's forward-sampled state."""
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import leaf_findings_codes

    m = get_example_model("pathfinder")
    ev, leaves, codes, nodes = leaf_findings_codes(m, 500, per_row=4, seed=7)
    assert leaves == sorted(v for v in m.nodes() if m.out_degree(v) == 0)
    assert ev.shape == (len(leaves), 500)
    assert ((ev != 255).sum(axis=0) == 4).all()
    rows = np.array([nodes.index(v) for v in leaves])
    obs = ev != 255
    assert (ev[obs] == codes[rows][obs]).all()
