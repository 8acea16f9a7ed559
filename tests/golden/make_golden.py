#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

This script is the only place that imports the read-only reference
(/root/reference, pgmpy 1.0.0).  It runs in the build container only; the
fixtures it writes (inputs + expected outputs, plain JSON / npz) are what the
tests and the oracle are pinned against on the GPU box, where the reference
does not exist.

    PYTHONHASHSEED=0 PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/make_golden.py [--only NAME ...] [--jobs 8]

Three offline shims under tests/golden/shims/ stand in for packages the image
lacks (scikit-base, statsmodels, opt_einsum).  opt_einsum's
greedy path is restated there; contraction values do not depend on the path
beyond floating-point rounding.

Fixture inventory (SURVEY.md §8(c) "Golden vectors"):
  networks/<net>_cpts.npz      CPT export of alarm / munin / pathfinder (parser pin)
  factor_ops.json              DiscreteFactor op results on seeded small factors
  unit_cases.json              hand-sized unit expectations of the reference tests
  alarm_queries.json           C1: HISTORY|CVP=LOW + 50 seeded query patterns (+ MAP)
  alarm_predict.json           predict / predict_probability on alarm rows (with NaN)
  alarm_predict_stochastic.json  predict(stochastic=True, seed=7) on duplicated alarm rows
  alarm_bp.npz / .json         BP calibration on a min-fill JT of alarm (full beliefs)
  munin_predict.npz            C3 template rows, MAP codes and marginals
  munin_c2_query.json          C2: 100 leaf findings -> 1 root posterior (row 0)
  munin_c2_rows.json           C2 on all 20 sampled rows: root + two joint=False sets
                               (+ munin_c2_mass: the root query's unnormalised joint per row)
  pathfinder_bp.npz / .json    C4: min-fill JT + beliefs (checksums) + marginals
"""
import argparse
import gzip
import json
import os
import random
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _setup():
    if os.environ.get("PYTHONHASHSEED") != "0":
        raise SystemExit("run with PYTHONHASHSEED=0 (product() orders variables by set hash)")
    for p in (REF, os.path.join(HERE, "shims")):
        if p not in sys.path:
            sys.path.insert(0, p)
    # the shims must shadow nothing real; put them after the reference
    sys.path.remove(os.path.join(HERE, "shims"))
    sys.path.insert(1, os.path.join(HERE, "shims"))
    import logging

    logging.getLogger("pgmpy").setLevel(logging.ERROR)
    from pgmpy import config

    config.set_show_progress(False) if hasattr(config, "set_show_progress") else None
    config.SHOW_PROGRESS = False


def _dump(name, obj):
    path = os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(obj, f, indent=None, separators=(",", ":"))
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def _model(name):
    from pgmpy.utils import get_example_model

    return get_example_model(name)


def _states(model):
    return {v: [str(s) for s in model.get_cpds(v).state_names[v]] for v in model.nodes()}


# ----------------------------------------------------------------------------- networks
def gen_networks():
    os.makedirs(os.path.join(HERE, "networks"), exist_ok=True)
    for net in ("alarm", "munin", "pathfinder"):
        m = _model(net)
        meta = {"nodes": [], "states": {}, "parents": {}}
        arrays = {}
        for i, v in enumerate(sorted(m.nodes())):
            cpd = m.get_cpds(v)
            meta["nodes"].append(v)
            meta["states"][v] = [str(s) for s in cpd.state_names[v]]
            meta["parents"][v] = list(cpd.variables[1:])
            meta.setdefault("parent_states", {})[v] = {
                p: [str(s) for s in cpd.state_names[p]] for p in cpd.variables[1:]
            }
            arrays[f"v{i}"] = np.asarray(cpd.values, dtype=np.float64).ravel()
        path = os.path.join(HERE, "networks", f"{net}_cpts.npz")
        np.savez_compressed(path, meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8), **arrays)
        print(f"wrote {path} ({os.path.getsize(path)} B)")


# ----------------------------------------------------------------------------- factor ops
def _fac_json(phi):
    return {
        "variables": list(phi.variables),
        "cardinality": [int(c) for c in phi.cardinality],
        "values": [float(x) for x in np.asarray(phi.values, dtype=np.float64).ravel()],
    }


def gen_factor_ops():
    """DiscreteFactor.{product,marginalize,maximize,reduce,normalize,divide,sum} on seeded factors.

    pgmpy/factors/discrete/DiscreteFactor.py:360-866."""
    from pgmpy.factors import factor_divide, factor_product
    from pgmpy.factors.discrete import DiscreteFactor

    rng = np.random.default_rng(20251017)
    names = [f"x{i}" for i in range(8)]
    cards = {n: int(c) for n, c in zip(names, rng.integers(2, 5, size=8))}
    cases = []

    def rand_factor(nv, zeros=False):
        vs = list(rng.choice(names, size=nv, replace=False))
        card = [cards[v] for v in vs]
        vals = rng.random(int(np.prod(card)))
        if zeros:
            vals[rng.random(vals.size) < 0.3] = 0.0
        return DiscreteFactor(vs, card, vals)

    for t in range(40):
        a = rand_factor(int(rng.integers(1, 4)), zeros=(t % 5 == 0))
        b = rand_factor(int(rng.integers(1, 4)), zeros=(t % 7 == 0))
        case = {"a": _fac_json(a), "b": _fac_json(b)}
        case["product"] = _fac_json(a.product(b, inplace=False))
        case["sum"] = _fac_json(a.sum(b, inplace=False))
        k = int(rng.integers(1, len(a.variables) + 1))
        mv = list(rng.choice(a.variables, size=k, replace=False))
        case["marg_vars"] = mv
        case["marginalize"] = _fac_json(a.marginalize(mv, inplace=False))
        case["maximize"] = _fac_json(a.maximize(mv, inplace=False))
        case["normalize"] = _fac_json(a.normalize(inplace=False))
        rv = list(rng.choice(a.variables, size=int(rng.integers(1, len(a.variables) + 1)), replace=False))
        red = [(v, int(rng.integers(0, cards[v]))) for v in rv]
        case["reduce_vals"] = red
        case["reduce"] = _fac_json(a.reduce(red, inplace=False))
        # divide needs scope(b) subset of scope(a): divide a by a marginal of a (with zeros)
        dsub = list(rng.choice(a.variables, size=int(rng.integers(1, len(a.variables) + 1)), replace=False))
        den = DiscreteFactor(dsub, [cards[v] for v in dsub], rng.random(int(np.prod([cards[v] for v in dsub]))))
        if t % 3 == 0:
            dv = den.values.ravel()
            dv[rng.random(dv.size) < 0.4] = 0.0
            den = DiscreteFactor(dsub, [cards[v] for v in dsub], dv)
        case["den"] = _fac_json(den)
        case["divide"] = _fac_json(a.divide(den, inplace=False))
        c = rand_factor(int(rng.integers(1, 3)))
        case["c"] = _fac_json(c)
        case["factor_product3"] = _fac_json(factor_product(a, b, c))
        case["argmax"] = int(np.argmax(a.values))
        cases.append(case)
    _dump("factor_ops.json", {"cards": cards, "cases": cases})


def gen_unit_cases():
    """Numbers the reference's own unit tests pin (test_Factor.py, test_ExactInference.py).

    Computed by running the reference on the same inputs as those tests."""
    from pgmpy.factors.discrete import DiscreteFactor, TabularCPD
    from pgmpy.inference import BeliefPropagation, VariableElimination
    from pgmpy.models import DiscreteBayesianNetwork, JunctionTree

    out = {}
    # test_Factor.py:390-450 marginalize; docstring examples DiscreteFactor.py:381-388
    phi = DiscreteFactor(["x1", "x2", "x3"], [2, 3, 2], range(12))
    out["marg_x1_x3"] = _fac_json(phi.marginalize(["x1", "x3"], inplace=False))
    phi1 = DiscreteFactor(["x1", "x2", "x3"], [2, 3, 2], range(12))
    phi2 = DiscreteFactor(["x3", "x4", "x1"], [2, 2, 2], range(8))
    out["product_doc"] = _fac_json(phi1.product(phi2, inplace=False))
    out["sum_doc"] = _fac_json(phi1.sum(phi2, inplace=False))
    d2 = DiscreteFactor(["x3", "x1"], [2, 2], range(1, 5))
    out["divide_doc"] = _fac_json(phi1.divide(d2, inplace=False))
    # divide with zeros: 0/0 -> 0, x/0 -> inf (test_Factor.py:674-723)
    num = DiscreteFactor(["x1", "x2"], [2, 2], [0.0, 1.0, 2.0, 0.0])
    den = DiscreteFactor(["x1"], [2], [0.0, 2.0])
    r = num.divide(den, inplace=False)
    out["divide_zero"] = {
        "variables": r.variables,
        "cardinality": [int(c) for c in r.cardinality],
        "values": [("inf" if np.isinf(x) else float(x)) for x in r.values.ravel()],
    }
    mx = DiscreteFactor(["x1", "x2", "x3"], [3, 2, 2],
                        [0.25, 0.35, 0.08, 0.16, 0.05, 0.07, 0.00, 0.00, 0.15, 0.21, 0.09, 0.18])
    out["maximize_doc"] = _fac_json(mx.maximize(["x2"], inplace=False))
    # TabularCPD normalize / marginalize / reduce docstring cases (CPD.py:449-567)
    cpd = TabularCPD("grade", 2, [[0.7, 0.2, 0.6, 0.2], [0.4, 0.4, 0.4, 0.8]], ["intel", "diff"], [2, 2])
    out["cpd_normalize"] = [list(map(float, r)) for r in cpd.normalize(inplace=False).get_values()]
    cpd2 = TabularCPD("grade", 2, [[0.7, 0.6, 0.6, 0.2], [0.3, 0.4, 0.4, 0.8]], ["intel", "diff"], [2, 2])
    out["cpd_marginalize_diff"] = [list(map(float, r)) for r in cpd2.marginalize(["diff"], inplace=False).get_values()]
    out["cpd_reduce_diff0"] = [list(map(float, r)) for r in cpd2.reduce([("diff", 0)], inplace=False).get_values()]

    # 6-node BN of test_ExactInference.py:22-60 (SAMIAM-pinned)
    bn = DiscreteBayesianNetwork([("A", "J"), ("R", "J"), ("J", "Q"), ("J", "L"), ("G", "L")])
    cpds = [
        TabularCPD("A", 2, [[0.2], [0.8]]),
        TabularCPD("R", 2, [[0.4], [0.6]]),
        TabularCPD("J", 2, [[0.9, 0.6, 0.7, 0.1], [0.1, 0.4, 0.3, 0.9]], ["R", "A"], [2, 2]),
        TabularCPD("Q", 2, [[0.9, 0.2], [0.1, 0.8]], ["J"], [2]),
        TabularCPD("L", 2, [[0.9, 0.45, 0.8, 0.1], [0.1, 0.55, 0.2, 0.9]], ["G", "J"], [2, 2]),
        TabularCPD("G", 2, [[0.6], [0.4]]),
    ]
    bn.add_cpds(*cpds)
    out["bn6"] = {
        "edges": [list(e) for e in bn.edges()],
        "cpds": [{"variable": c.variable, "card": int(c.variable_card),
                  "values": [list(map(float, r)) for r in c.get_values()],
                  "evidence": list(c.variables[1:]), "evidence_card": [int(x) for x in c.cardinality[1:]]}
                 for c in cpds],
    }
    ve = VariableElimination(bn)
    q = {}
    for order in ("greedy", "MinFill", "MinNeighbors", "MinWeight", "WeightedMinFill"):
        r1 = ve.query(["J"], show_progress=False, elimination_order=order)
        r2 = ve.query(["J", "Q"], evidence={"A": 0, "R": 0, "G": 0, "L": 1}, show_progress=False,
                      elimination_order=order)
        r3 = ve.query(["Q", "J"], evidence={"A": 1}, joint=False, show_progress=False, elimination_order=order)
        q[order] = {"J": _fac_json(r1), "JQ|ARGL": _fac_json(r2),
                    "Q,J|A=1 sep": {k: _fac_json(v) for k, v in r3.items()}}
    out["bn6_queries"] = q
    out["bn6_map_J"] = ve.map_query(["J"], show_progress=False)
    out["bn6_map_JQ"] = ve.map_query(["J", "Q"], evidence={"A": 0, "R": 0, "G": 0, "L": 1}, show_progress=False)
    out["bn6_max_marginal"] = float(ve.max_marginal(["J", "Q"], evidence={"A": 0, "R": 0, "G": 0, "L": 1}))
    bp = BeliefPropagation(bn)
    out["bn6_bp_query"] = _fac_json(bp.query(["J", "Q"], evidence={"A": 0, "R": 0, "G": 0, "L": 1}, show_progress=False))
    out["bn6_bp_map"] = bp.map_query(["J", "Q"], evidence={"A": 0, "R": 0, "G": 0, "L": 1}, show_progress=False)

    # BP on a given 3-clique junction tree (test_ExactInference.py:891-1033)
    jt = JunctionTree()
    jt.add_edges_from([(("A", "B"), ("B", "C")), (("B", "C"), ("C", "D"))])
    phi1 = DiscreteFactor(["A", "B"], [2, 3], range(6))
    phi2 = DiscreteFactor(["B", "C"], [3, 2], range(6))
    phi3 = DiscreteFactor(["C", "D"], [2, 2], range(4))
    jt.add_factors(phi1, phi2, phi3)
    bpj = BeliefPropagation(jt)
    bpj.calibrate()
    out["jt3"] = {
        "cliques": [list(c) for c in jt.nodes()],
        "edges": [[list(a), list(b)] for a, b in jt.edges()],
        "factors": [_fac_json(f) for f in (phi1, phi2, phi3)],
        "clique_beliefs": [[list(c), _fac_json(v)] for c, v in bpj.get_clique_beliefs().items()],
        "sepset_beliefs": [[sorted(map(list, k)), _fac_json(v)] for k, v in bpj.get_sepset_beliefs().items()],
    }
    bpj2 = BeliefPropagation(jt)
    bpj2.max_calibrate()
    out["jt3_max"] = {
        "clique_beliefs": [[list(c), _fac_json(v)] for c, v in bpj2.get_clique_beliefs().items()],
    }
    _dump("unit_cases.json", out)


# ----------------------------------------------------------------------------- alarm
def gen_alarm():
    """C1: HISTORY|CVP=LOW plus 50 patterns from random.Random(1)."""
    from pgmpy.inference import VariableElimination
    from pgmpy.sampling import BayesianModelSampling

    m = _model("alarm")
    ve = VariableElimination(m)
    res = {"history_cvp_low": _fac_json(ve.query(["HISTORY"], {"CVP": "LOW"}, show_progress=False))}
    samples = BayesianModelSampling(m).forward_sample(size=50, seed=1, show_progress=False)
    rng = random.Random(1)
    nodes = sorted(m.nodes())
    pats = []
    for i in range(50):
        picks = rng.sample(nodes, 8)
        qv, ev = picks[:3], picks[3:]
        evidence = {v: str(samples.iloc[i][v]) for v in ev}
        r = ve.query(qv, evidence, joint=False, show_progress=False)
        rj = ve.query(qv, evidence, joint=True, show_progress=False)
        rm = ve.query(qv, evidence, joint=True, show_progress=False, elimination_order="MinFill")
        mp = ve.map_query(qv, evidence, show_progress=False)
        jv = np.asarray(rj.values).ravel()
        srt = np.sort(jv)[::-1]
        pats.append({
            "variables": qv, "evidence": evidence,
            "marginals": {k: _fac_json(v) for k, v in r.items()},
            "joint": _fac_json(rj), "joint_minfill": _fac_json(rm),
            "map": {k: str(v) for k, v in mp.items()},
            "map_gap": float(srt[0] - srt[1]) if srt.size > 1 else 1.0,
        })
    res["patterns"] = pats
    _dump("alarm_queries.json", res)


def gen_alarm_predict():
    """predict / predict_probability (DiscreteBayesianNetwork.py:731-989) on alarm rows."""
    import pandas as pd
    from pgmpy.sampling import BayesianModelSampling

    m = _model("alarm")
    df = BayesianModelSampling(m).forward_sample(size=300, seed=3, show_progress=False)
    rng = np.random.default_rng(3)
    missing = ["LVFAILURE", "HYPOVOLEMIA", "STROKEVOLUME"]
    data = df.drop(columns=missing).astype(object)
    # sprinkle NaNs into 30 rows (these rows predict extra variables)
    nan_rows = rng.choice(len(data), size=30, replace=False)
    nan_col_choices = ["HISTORY", "CVP", "PCWP"]
    for r in nan_rows:
        data.iat[r, data.columns.get_loc(nan_col_choices[r % 3])] = np.nan
    pred = m.predict(data, n_jobs=1)
    clean = data.drop(index=data.index[nan_rows])
    prob = m.predict_probability(clean)
    _dump("alarm_predict.json", {
        "columns": list(data.columns),
        "rows": [[None if (isinstance(x, float) and np.isnan(x)) else str(x) for x in row] for row in data.values],
        "missing": missing,
        "predict_columns": list(pred.columns),
        "predict": [[None if (isinstance(x, float) and np.isnan(x)) else str(x) for x in row] for row in pred.values],
        "prob_index": [int(i) for i in clean.index],
        "prob_columns": list(prob.columns),
        "prob": prob.values.tolist(),
    })


def gen_alarm_predict_stochastic():
    """predict(stochastic=True, seed=...) (DiscreteBayesianNetwork.py:866-910): duplicated rows (the
    reference draws len(group) samples per unique row, each group from a fresh Generator(seed)).
    Case "one": a single missing variable (factor order is trivial).  Case "two": two missing
    variables and NaN cells (extra query variables); its factor order follows set iteration under
    PYTHONHASHSEED=0, so the test replays it in a PYTHONHASHSEED=0 subprocess."""
    import pandas as pd
    from pgmpy.sampling import BayesianModelSampling

    m = _model("alarm")
    df = BayesianModelSampling(m).forward_sample(size=60, seed=11, show_progress=False)
    rng = np.random.default_rng(11)
    picks = np.concatenate([np.arange(40), rng.choice(40, size=35)])
    rng.shuffle(picks)
    out = {"seed": 7}
    for case, missing, nan_col in (("one", ["LVFAILURE"], None), ("two", ["HYPOVOLEMIA", "STROKEVOLUME"], "CVP")):
        data = df.iloc[picks].drop(columns=missing).astype(object).reset_index(drop=True)
        if nan_col is not None:
            for r in range(0, len(data), 9):
                data.iat[r, data.columns.get_loc(nan_col)] = np.nan
        pred = m.predict(data, stochastic=True, seed=7, n_jobs=1)
        out[case] = {
            "columns": list(data.columns),
            "rows": [[None if (isinstance(x, float) and np.isnan(x)) else str(x) for x in row] for row in data.values],
            "missing": missing,
            "predict_columns": list(pred.columns),
            "predict": [[None if (isinstance(x, float) and np.isnan(x)) else str(x) for x in row] for row in pred.values],
        }
    _dump("alarm_predict_stochastic.json", out)


# ----------------------------------------------------------------------------- junction trees
def minfill_junction_tree(model):
    """Min-fill JT used as the BP oracle input (SURVEY.md §8(c) "BP oracle caveat")."""
    import networkx as nx
    from networkx.algorithms.approximation import treewidth_min_fill_in
    from pgmpy.factors.discrete import DiscreteFactor
    from pgmpy.models import JunctionTree
    from pgmpy.factors import factor_product

    moral = model.moralize()
    g = nx.Graph(moral.edges())
    g.add_nodes_from(model.nodes())
    tw, decomp = treewidth_min_fill_in(g)
    bags = [tuple(sorted(b)) for b in decomp.nodes()]
    jt = JunctionTree()
    if len(bags) == 1:
        jt.add_node(bags[0])
    for a, b in decomp.edges():
        jt.add_edge(tuple(sorted(a)), tuple(sorted(b)))
    assigned = {b: [] for b in bags}
    for node in sorted(model.nodes()):
        cpd = model.get_cpds(node)
        scope = set(cpd.scope())
        for b in bags:
            if scope <= set(b):
                assigned[b].append(cpd.to_factor())
                break
        else:
            raise RuntimeError(f"no bag covers {node}")
    card = model.get_cardinality()
    factors = []
    for b in bags:
        ones = DiscreteFactor(list(b), [card[v] for v in b], np.ones(int(np.prod([card[v] for v in b]))),
                              state_names={v: model.get_cpds(v).state_names[v] for v in b})
        pot = factor_product(ones, *assigned[b]) if assigned[b] else ones
        pot = DiscreteFactor(list(b), [card[v] for v in b],
                             pot.values.transpose([pot.variables.index(v) for v in b]).ravel(),
                             state_names={v: model.get_cpds(v).state_names[v] for v in b})
        factors.append(pot)
    jt.add_factors(*factors)
    return jt, bags, [(tuple(sorted(a)), tuple(sorted(b))) for a, b in decomp.edges()], assigned


def _aligned(phi, order):
    return np.asarray(phi.values).transpose([phi.variables.index(v) for v in order])


def _bp_case(model, jt, bags, evidence):
    """Calibrate with evidence applied as 0/1 indicators into the first clique holding each var."""
    import copy

    from pgmpy.factors.discrete import DiscreteFactor
    from pgmpy.inference import BeliefPropagation

    jt = copy.deepcopy(jt)
    card = model.get_cardinality()
    states = _states(model)
    for var, st in evidence.items():
        for b in bags:
            if var in b:
                f = jt.get_factors(b)
                ind = np.zeros(card[var])
                ind[states[var].index(st)] = 1.0
                f2 = f.product(DiscreteFactor([var], [card[var]], ind,
                                              state_names={var: model.get_cpds(var).state_names[var]}),
                               inplace=False)
                f2 = DiscreteFactor(list(b), [card[v] for v in b], _aligned(f2, b).ravel(), state_names=f.state_names)
                jt.remove_factors(f)
                jt.add_factors(f2)
                break
    bp = BeliefPropagation(jt)
    bp.calibrate()
    cb = bp.get_clique_beliefs()
    sb = bp.get_sepset_beliefs()
    beliefs = {b: _aligned(cb[b], b).ravel() for b in bags}
    seps = {}
    for k, v in sb.items():
        a, b = sorted(tuple(x) for x in k)
        sep = tuple(sorted(set(a) & set(b)))
        seps[(a, b)] = _aligned(v, sep).ravel()
    # variable marginals from the first clique holding each variable
    marg = {}
    for var in sorted(model.nodes()):
        for b in bags:
            if var in b:
                arr = beliefs[b].reshape([card[v] for v in b])
                axes = tuple(i for i, v in enumerate(b) if v != var)
                m = arr.sum(axis=axes)
                marg[var] = (m / m.sum()).tolist()
                break
    return beliefs, seps, marg


def gen_alarm_bp():
    m = _model("alarm")
    jt, bags, edges, _ = minfill_junction_tree(m)
    from pgmpy.sampling import BayesianModelSampling

    s = BayesianModelSampling(m).forward_sample(size=4, seed=7, show_progress=False)
    leaves = sorted(n for n in m.nodes() if m.out_degree(n) == 0)
    rng = random.Random(7)
    cases = [{}]
    for i in range(3):
        ev = rng.sample(leaves, 4)
        cases.append({v: str(s.iloc[i][v]) for v in ev})
    arrays, meta = {}, {"bags": [list(b) for b in bags], "edges": [[list(a), list(b)] for a, b in edges],
                        "cases": []}
    for ci, ev in enumerate(cases):
        beliefs, seps, marg = _bp_case(m, jt, bags, ev)
        for bi, b in enumerate(bags):
            arrays[f"c{ci}_b{bi}"] = beliefs[b]
        sep_keys = []
        for si, (k, v) in enumerate(sorted(seps.items())):
            arrays[f"c{ci}_s{si}"] = v
            sep_keys.append([list(k[0]), list(k[1])])
        meta["cases"].append({"evidence": ev, "sep_keys": sep_keys, "marginals": marg})
    np.savez_compressed(os.path.join(HERE, "alarm_bp.npz"), **arrays)
    _dump("alarm_bp.json", meta)


def gen_pathfinder_bp():
    """C4: min-fill JT, 0 and 4-finding calibrations, checksums + marginals."""
    m = _model("pathfinder")
    jt, bags, edges, _ = minfill_junction_tree(m)
    from pgmpy.sampling import BayesianModelSampling

    s = BayesianModelSampling(m).forward_sample(size=4, seed=7, show_progress=False)
    leaves = sorted(n for n in m.nodes() if m.out_degree(n) == 0)
    rng = random.Random(7)
    cases = [{}]
    for i in range(2):
        ev = rng.sample(leaves, 4)
        cases.append({v: str(s.iloc[i][v]) for v in ev})
    wrng = np.random.default_rng(123)
    arrays = {}
    meta = {"bags": [list(b) for b in bags], "edges": [[list(a), list(b)] for a, b in edges], "cases": []}
    sizes = [len(_aligned_size(m, b)) if False else None for b in bags]
    card = m.get_cardinality()
    bag_sizes = [int(np.prod([card[v] for v in b])) for b in bags]
    small = sorted(range(len(bags)), key=lambda i: bag_sizes[i])[:12]
    for ci, ev in enumerate(cases):
        t0 = time.time()
        beliefs, seps, marg = _bp_case(m, jt, bags, ev)
        cs = []
        for bi, b in enumerate(bags):
            x = beliefs[b]
            w = np.random.default_rng(1000 + bi).random(x.size)
            cs.append([float(x.sum()), float((w * x).sum())])
        arrays[f"c{ci}_checksums"] = np.array(cs)
        for bi in small:
            arrays[f"c{ci}_b{bi}"] = beliefs[bags[bi]]
        meta["cases"].append({"evidence": ev, "marginals": marg, "seconds": time.time() - t0})
    meta["small_bags"] = small
    np.savez_compressed(os.path.join(HERE, "pathfinder_bp.npz"), **arrays)
    _dump("pathfinder_bp.json", meta)


def _aligned_size(m, b):
    return b


# ----------------------------------------------------------------------------- munin
MUNIN_MISSING = None


def _munin_rows(n, seed=42):
    from pgmpy.sampling import BayesianModelSampling

    m = _model("munin")
    return m, BayesianModelSampling(m).forward_sample(size=n, seed=seed, show_progress=False)


def _munin_worker(args):
    _setup()
    lo, hi, rows_json, missing = args
    import pandas as pd

    m = _model("munin")
    df = pd.DataFrame(rows_json)
    df = df.iloc[lo:hi]
    t0 = time.time()
    pred = m.predict(df, n_jobs=1)
    t1 = time.time()
    prob = m.predict_probability(df)
    t2 = time.time()
    return lo, pred[missing].values.tolist(), list(prob.columns), prob.values.tolist(), t1 - t0, t2 - t1


def gen_munin_predict(n_rows=1000, jobs=8):
    """C3 template: missing = random.Random(0).sample(sorted(nodes), 3)."""
    m, samples = _munin_rows(n_rows, seed=42)
    nodes = sorted(m.nodes())
    missing = random.Random(0).sample(nodes, 3)
    print("munin missing:", missing)
    df = samples.drop(columns=missing).astype(str)
    rows_json = df.to_dict(orient="list")
    chunks = []
    step = (n_rows + jobs - 1) // jobs
    for lo in range(0, n_rows, step):
        chunks.append((lo, min(n_rows, lo + step), rows_json, missing))
    with Pool(jobs) as pool:
        res = pool.map(_munin_worker, chunks)
    res.sort()
    states = _states(m)
    pred_codes = np.array([[states[v].index(str(x)) for v, x in zip(missing, r)] for _, p, _, _, _, _ in res for r in p],
                          dtype=np.uint8)
    prob_cols = res[0][2]
    prob = np.array([r for _, _, _, p, _, _ in res for r in p], dtype=np.float64)
    cols = list(df.columns)
    codes = np.array([[states[c].index(str(x)) for x in df[c]] for c in cols], dtype=np.uint8)  # [V][N]
    meta = {"missing": missing, "columns": cols, "prob_columns": prob_cols,
            "predict_s_per_row": sum(r[4] for r in res) / n_rows,
            "predict_probability_s_per_row": sum(r[5] for r in res) / n_rows}
    np.savez_compressed(os.path.join(HERE, "munin_predict.npz"), codes=codes, map_codes=pred_codes, prob=prob,
                        meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8))
    print("wrote munin_predict.npz", meta["predict_s_per_row"], meta["predict_probability_s_per_row"])


def gen_munin_c2():
    """C2: 100 leaf findings -> 1 root, VariableElimination.query greedy path."""
    from pgmpy.inference import VariableElimination

    m, samples = _munin_rows(20, seed=0)
    leaves = sorted(n for n in m.nodes() if m.out_degree(n) == 0)
    roots = sorted(n for n in m.nodes() if m.in_degree(n) == 0)
    rng = random.Random(100000)
    E = rng.sample(leaves, 100)
    q = [rng.choice(roots)]
    evidence = {v: str(samples.iloc[0][v]) for v in E}
    t0 = time.time()
    r = VariableElimination(m).query(q, evidence, show_progress=False)
    dt = time.time() - t0
    _dump("munin_c2_query.json", {"variables": q, "evidence": evidence, "result": _fac_json(r), "seconds": dt})


def _c2_pattern():
    """The C2 evidence pattern: the same 100 leaf findings E and root q as gen_munin_c2, plus two
    joint=False query sets of non-root variables (a node with its parent / children in munin's nerve
    chains). They were picked among 100 seeded local sets by the reference's own greedy path cost
    (<= 1e10 multiply-adds, <= 3.6e7-entry intermediates, so each query takes ~1 min here); a random
    4-variable set costs ~4e11 (~30 min per query)."""
    m, samples = _munin_rows(20, seed=0)
    leaves = sorted(n for n in m.nodes() if m.out_degree(n) == 0)
    roots = sorted(n for n in m.nodes() if m.in_degree(n) == 0)
    rng = random.Random(100000)
    E = rng.sample(leaves, 100)
    q = [rng.choice(roots)]
    qms = [["R_MEDD2_SALOSS", "R_DIFFN_LNLW_MEDD2_SALOSS", "R_MEDD2_DSLOW_EW", "R_MEDD2_EFFAXLOSS"],
           ["L_MEDD2_DISP_EW", "L_DIFFN_MEDD2_DISP", "L_MEDD2_DISP_EWD"]]
    return m, samples, E, q, qms


def _c2_row_worker(i):
    _setup()
    from pgmpy.inference import VariableElimination

    m, samples, E, q, qms = _c2_pattern()
    evidence = {v: str(samples.iloc[i][v]) for v in E}
    ve = VariableElimination(m)
    out = {"row": i, "evidence": evidence, "separate": [], "seconds": []}
    t0 = time.time()
    out["root"] = _fac_json(ve.query(q, evidence, show_progress=False))
    out["seconds"].append(time.time() - t0)
    for qm in qms:
        t0 = time.time()
        sep = ve.query(qm, evidence, joint=False, show_progress=False)
        out["seconds"].append(time.time() - t0)
        out["separate"].append({k: _fac_json(v) for k, v in sep.items()})
    return out


def gen_munin_c2_rows(jobs=6, rows=20):
    """C2 on every row of forward_sample(size=20, seed=0): the same 100 findings and root as
    munin_c2_query.json (one evidence pattern, one compiled plan per query) -> the root posterior, and
    two joint=False queries over 3-4 non-root variables (ExactInference.py:349-440, greedy path; the
    per-variable results are marginalize + normalize of the joint, L423-432)."""
    _, _, E, q, qms = _c2_pattern()
    with Pool(jobs) as pool:
        res = pool.map(_c2_row_worker, list(range(rows)), chunksize=1)
    res.sort(key=lambda r: r["row"])
    _dump("munin_c2_rows.json", {"variables": q, "separate_variables": qms, "evidence_variables": E, "rows": res})


def _c2_mass_worker(i):
    """Row i's root query through the reference, recording what its contract call returns: the
    pruned, evidence-sliced sum-product (ExactInference.py:404-406) BEFORE normalize (L420)."""
    _setup()
    import pgmpy.inference.ExactInference as XI
    from pgmpy.inference import VariableElimination

    m, samples, E, q, _ = _c2_pattern()
    evidence = {v: str(samples.iloc[i][v]) for v in E}
    seen = []
    contract = XI.contract

    def recording_contract(*a, **k):
        r = contract(*a, **k)
        seen.append(np.array(r, dtype=np.float64, copy=True))
        return r

    XI.contract = recording_contract
    try:
        t0 = time.time()
        post = VariableElimination(m).query(q, evidence, show_progress=False)
        dt = time.time() - t0
    finally:
        XI.contract = contract
    assert len(seen) == 1, len(seen)
    return {"row": i, "root_unnormalized": [float(x) for x in seen[0].ravel()],
            "root": [float(x) for x in np.asarray(post.values).ravel()], "seconds": dt}


def gen_munin_c2_mass(jobs=6):
    """the C2 root posterior is one-hot on all 20 rows, so its normalised value pins
    only the support.  Add to every row of munin_c2_rows.json the root query's unnormalised joint
    (the reference's contract output before normalize: P(root, findings) over the pruned model,
    inference/base.py:154-212 + ExactInference.py:349-406) as `root_unnormalized`."""
    path = os.path.join(HERE, "munin_c2_rows.json")
    with open(path) as f:
        g = json.load(f)
    with Pool(jobs) as pool:
        res = pool.map(_c2_mass_worker, list(range(len(g["rows"]))), chunksize=1)
    for r in res:
        row = g["rows"][r["row"]]
        assert np.allclose(r["root"], row["root"]["values"], rtol=1e-12, atol=0), r["row"]
        row["root_unnormalized"] = r["root_unnormalized"]
        row["seconds"].append(r["seconds"])
    _dump("munin_c2_rows.json", g)


# ----------------------------------------------------------------------------- small API completion
def gen_api_extras():
    """DiscreteBayesianNetwork.get_state_probability (DiscreteBayesianNetwork.py:991-1041;
    the reference enumerates every combination of the unassigned variables, so alarm cases leave at most
    6 of its 37 unassigned), TabularCPD.reorder_parents (CPD.py:598-727) and to_dataframe (CPD.py:336-410)."""
    from pgmpy.factors.discrete import TabularCPD

    out = {"state_probability": [], "reorder_parents": [], "to_dataframe": []}
    asia = _model("asia")
    cases = [("asia", {"either": "no", "tub": "no", "xray": "yes", "bronc": "no"}),
             ("asia", {"smoke": "yes"}), ("asia", {"lung": "yes", "dysp": "no"}),
             ("asia", {v: str(asia.states[v][i % len(asia.states[v])]) for i, v in enumerate(sorted(asia.nodes()))})]
    alarm = _model("alarm")
    rng = random.Random(5)
    from pgmpy.sampling import BayesianModelSampling

    samples = BayesianModelSampling(alarm).forward_sample(size=4, seed=3, show_progress=False)
    nodes = sorted(alarm.nodes())
    for k in range(4):
        keep = rng.sample(nodes, len(nodes) - (6 if k < 3 else 0))
        row = samples.iloc[k]
        cases.append(("alarm", {v: str(row[v]) for v in keep}))
    for net, st in cases:
        m = asia if net == "asia" else alarm
        t0 = time.time()
        p = m.get_state_probability(st)
        out["state_probability"].append({"network": net, "states": st, "probability": float(p),
                                         "seconds": time.time() - t0})
        print(net, len(st), p)
    errs = []
    for st in ({"nope": "yes"}, {"smoke": "maybe"}):
        try:
            asia.get_state_probability(st)
        except ValueError as e:
            errs.append({"states": st, "error": "ValueError", "message": str(e)})
    out["state_probability_errors"] = errs
    # reorder_parents: the reference's docstring CPD and an alarm CPD with 4 parents, inplace and not
    grade = dict(variable="grade", variable_card=3,
                 values=[[0.1, 0.1, 0.0, 0.4, 0.2, 0.1], [0.3, 0.2, 0.1, 0.4, 0.3, 0.2], [0.6, 0.7, 0.9, 0.2, 0.5, 0.7]],
                 evidence=["diff", "intel"], evidence_card=[2, 3])
    big = alarm.get_cpds("CATECHOL")
    for spec, order in ((grade, ["intel", "diff"]), (None, list(reversed(big.variables[1:])))):
        for inplace in (False, True):
            cpd = TabularCPD(**spec) if spec else big.copy()
            before = {"variable": cpd.variable, "variable_card": int(cpd.variable_card),
                      "values": np.asarray(cpd.get_values()).tolist(), "evidence": list(cpd.variables[1:]),
                      "evidence_card": [int(c) for c in cpd.cardinality[1:]],
                      "state_names": {k: [str(x) for x in v] for k, v in cpd.state_names.items()}}
            r = cpd.reorder_parents(order, inplace=inplace)
            out["reorder_parents"].append({
                "cpd": before, "new_order": order, "inplace": inplace, "returned": np.asarray(r).tolist(),
                "variables_after": list(cpd.variables), "cardinality_after": [int(c) for c in cpd.cardinality],
                "values_after": np.asarray(cpd.values).ravel().tolist(),
                "state_names_after": {k: [str(x) for x in v] for k, v in cpd.state_names.items()}})
    try:
        TabularCPD(**grade).reorder_parents(["intel"])
    except ValueError as e:
        out["reorder_parents_error"] = str(e)
    for node in ("HISTORY", "CATECHOL", "HR"):
        df = alarm.get_cpds(node).to_dataframe()
        out["to_dataframe"].append({"node": node, "columns": [str(c) for c in df.columns],
                                    "columns_name": str(df.columns.name),
                                    "index_names": [str(n) for n in df.index.names],
                                    "index": [[str(x) for x in (t if isinstance(t, tuple) else (t,))] for t in df.index],
                                    "values": df.to_numpy().tolist()})
    _dump("api_extras.json", out)


# ----------------------------------------------------------------------------- Markov networks
def _sorted_fac(phi):
    """A factor as {variables sorted, values aligned to them} (hash-order independent)."""
    order = sorted(phi.variables)
    vals = np.asarray(phi.values, dtype=np.float64).transpose([phi.variables.index(v) for v in order])
    return {"variables": order, "cardinality": [int(c) for c in vals.shape],
            "values": [float(x) for x in vals.ravel()]}


def _markov_case(mm, queries, maps, max_marginals, orders=None, bp=True, bp_queries=()):
    """Run the reference on a DiscreteMarkovNetwork: VE greedy / explicit-order queries, map_query,
    max_marginal, partition function, to_junction_tree structure, BP calibration and BP queries."""
    from pgmpy.inference import BeliefPropagation, VariableElimination

    ve = VariableElimination(mm)
    out = {"nodes": sorted(mm.nodes()), "edges": sorted(sorted(e) for e in mm.edges()),
           "factors": [_fac_json(f) for f in mm.factors], "queries": [], "maps": [], "max_marginals": []}
    for variables, evidence in queries:
        rec = {"variables": variables, "evidence": evidence,
               "joint": _fac_json(ve.query(variables, evidence, show_progress=False)),
               "separate": {k: _fac_json(v) for k, v in
                            ve.query(variables, evidence, joint=False, show_progress=False).items()}}
        if orders is not None:
            elim = [v for v in orders if v not in variables and v not in evidence]
            rec["order"] = elim
            rec["joint_order"] = _fac_json(ve.query(variables, evidence, elimination_order=elim,
                                                    show_progress=False))
        out["queries"].append(rec)
    for variables, evidence in maps:
        r = ve.map_query(variables, evidence, show_progress=False)
        out["maps"].append({"variables": variables, "evidence": evidence, "result": {k: str(v) for k, v in r.items()}})
    for variables, evidence in max_marginals:
        out["max_marginals"].append({"variables": variables, "evidence": evidence,
                                     "result": float(ve.max_marginal(variables, evidence, show_progress=False))})
    out["partition_function"] = float(mm.get_partition_function())
    jt = mm.to_junction_tree()
    out["jt_cliques"] = sorted(sorted(c) for c in jt.nodes())
    out["jt_edges"] = sorted(sorted([sorted(a), sorted(b)]) for a, b in jt.edges())
    if bp:
        b = BeliefPropagation(mm)
        b.calibrate()
        out["bp_clique_beliefs"] = sorted(([sorted(c), _sorted_fac(v)] for c, v in b.get_clique_beliefs().items()),
                                          key=lambda x: x[0])
        out["bp_sepset_beliefs"] = sorted(([sorted(sorted(x) for x in k), _sorted_fac(v)]
                                           for k, v in b.get_sepset_beliefs().items()), key=lambda x: x[0])
        b2 = BeliefPropagation(mm)
        b2.max_calibrate()
        out["bp_max_clique_beliefs"] = sorted(([sorted(c), _sorted_fac(v)]
                                               for c, v in b2.get_clique_beliefs().items()), key=lambda x: x[0])
        out["bp_queries"] = []
        for variables, evidence in bp_queries:
            b3 = BeliefPropagation(mm)
            q = b3.query(variables, evidence, show_progress=False)
            m = BeliefPropagation(mm).map_query(variables, evidence, show_progress=False)
            out["bp_queries"].append({"variables": variables, "evidence": evidence, "joint": _fac_json(q),
                                      "map": {k: str(v) for k, v in m.items()}})
    return out


def gen_markov():
    """DiscreteMarkovNetwork container, triangulation, junction tree and VE / BP over it
    (pgmpy/models/DiscreteMarkovNetwork.py:16-882; test_ExactInference.py:639-889,
    test_DiscreteMarkovNetwork.py:246-591)."""
    from pgmpy.factors.discrete import DiscreteFactor, TabularCPD
    from pgmpy.inference import VariableElimination
    from pgmpy.models import DiscreteMarkovNetwork, FactorGraph

    out = {}
    # test_ExactInference.py:659-699: the moralised 6-node BN as a Markov network (SAMIAM values)
    mm = DiscreteMarkovNetwork([("A", "J"), ("R", "J"), ("J", "Q"), ("J", "L"), ("G", "L"), ("A", "R"), ("J", "G")])
    mm.add_factors(
        TabularCPD("A", 2, values=[[0.2], [0.8]]).to_factor(),
        TabularCPD("R", 2, values=[[0.4], [0.6]]).to_factor(),
        TabularCPD("J", 2, values=[[0.9, 0.6, 0.7, 0.1], [0.1, 0.4, 0.3, 0.9]], evidence=["A", "R"],
                   evidence_card=[2, 2]).to_factor(),
        TabularCPD("Q", 2, values=[[0.9, 0.2], [0.1, 0.8]], evidence=["J"], evidence_card=[2]).to_factor(),
        TabularCPD("L", 2, values=[[0.9, 0.45, 0.8, 0.1], [0.1, 0.55, 0.2, 0.9]], evidence=["J", "G"],
                   evidence_card=[2, 2]).to_factor(),
        TabularCPD("G", 2, [[0.6], [0.4]]).to_factor())
    queries = [(["J"], {}), (["Q", "J"], {}), (["J"], {"A": 0, "R": 1}), (["J", "Q"], {"A": 0, "R": 0, "G": 0, "L": 1}),
               (["L", "A"], {"Q": 1})]
    maps = [([], {}), (["A", "R", "L"], {"J": 0, "Q": 1, "G": 0}), (["J"], {"L": 1})]
    mms = [([], None), (["G"], None), (["G", "R"], None), (["G", "R", "A"], None), (["J"], {"L": 1})]
    out["markov6"] = _markov_case(mm, queries, maps, mms, orders=["G", "Q", "A", "J", "L", "R"],
                                  bp_queries=[(["J"], {}), (["J", "Q"], {"A": 0, "R": 0, "G": 0, "L": 1})])
    ve = VariableElimination(mm)
    ig = ve.induced_graph(["G", "Q", "A", "J", "L", "R"])
    out["markov6"]["induced_graph"] = sorted(sorted(e) for e in ig.edges())
    out["markov6"]["induced_width"] = int(ve.induced_width(["G", "Q", "A", "J", "L", "R"]))
    out["markov6"]["triangulations"] = {
        h: sorted(sorted(e) for e in mm.triangulate(heuristic=h).edges()) for h in ("H1", "H2", "H3", "H4", "H5", "H6")}

    # test_ExactInference.py:639-656: duplicated (identical-valued) factors
    dup = DiscreteMarkovNetwork([("A", "B"), ("A", "C")])
    dup.add_factors(DiscreteFactor(["A", "B"], [2, 2], np.eye(2) * 2), DiscreteFactor(["A", "C"], [2, 2], np.eye(2) * 2))
    out["duplicated"] = {"factors": [_fac_json(f) for f in dup.factors], "edges": [["A", "B"], ["A", "C"]],
                         "query_A": _fac_json(VariableElimination(dup).query(["A"], show_progress=False))}

    # test_DiscreteMarkovNetwork.py:246-259, 421-591: the 4-cycle with cardinalities 2/3/4/5
    rng = np.random.default_rng(4242)
    cyc = DiscreteMarkovNetwork([("a", "b"), ("b", "c"), ("c", "d"), ("d", "a")])
    cyc.add_factors(DiscreteFactor(["a", "b"], [2, 3], rng.random(6)), DiscreteFactor(["b", "c"], [3, 4], rng.random(12)),
                    DiscreteFactor(["c", "d"], [4, 5], rng.random(20)), DiscreteFactor(["d", "a"], [5, 2], rng.random(10)))
    out["cycle4"] = _markov_case(cyc, [(["a"], {}), (["b", "d"], {"c": 2})], [(["a", "c"], {})], [([], None)],
                                 orders=["a", "b", "c", "d"], bp_queries=[(["b"], {"a": 1})])
    out["cycle4"]["triangulations"] = {
        h: sorted(sorted(e) for e in cyc.triangulate(heuristic=h).edges()) for h in ("H1", "H2", "H3", "H4", "H5", "H6")}

    # a seeded random pairwise + triangle Markov network (12 variables, cardinalities 2-4)
    rng = np.random.default_rng(777)
    names = [f"v{i:02d}" for i in range(12)]
    card = {n: int(c) for n, c in zip(names, rng.integers(2, 5, size=12))}
    edges = set()
    for i in range(1, 12):  # a random spanning tree ...
        edges.add(tuple(sorted((names[i], names[int(rng.integers(0, i))]))))
    while len(edges) < 20:  # ... plus chords
        a, b = rng.choice(12, size=2, replace=False)
        edges.add(tuple(sorted((names[a], names[b]))))
    edges = sorted(edges)
    rnd = DiscreteMarkovNetwork(edges)
    facs = [DiscreteFactor([a, b], [card[a], card[b]], rng.random(card[a] * card[b]) + 0.05) for a, b in edges]
    adj = {n: set() for n in names}
    for a, b in edges:
        adj[a].add(b)
        adj[b].add(a)
    tri = sorted({tuple(sorted((a, b, c))) for a, b in edges for c in adj[a] & adj[b]})[:3]
    for t in tri:
        facs.append(DiscreteFactor(list(t), [card[v] for v in t], rng.random(int(np.prod([card[v] for v in t])))))
    rnd.add_factors(*facs)
    queries = [([names[0]], {}), ([names[3], names[7]], {names[1]: 1, names[10]: 0}),
               ([names[5], names[11], names[2]], {names[8]: 1})]
    out["random12"] = _markov_case(rnd, queries, [([names[4], names[9]], {names[0]: 1})],
                                   [([names[6]], {names[3]: 0})], orders=list(reversed(names)),
                                   bp_queries=[([names[3]], {names[1]: 1}), ([names[5], names[6]], {})])
    # the heuristic scores of this network tie (cardinalities 2-4), and the reference breaks ties by
    # set iteration order (string hashes): pin the fill-in of an explicit order instead
    out["random12"]["order_triangulation"] = {
        "order": names[::2] + names[1::2],
        "edges": sorted(sorted(e) for e in rnd.triangulate(order=names[::2] + names[1::2]).edges())}

    # the alarm network as a Markov network (to_markov_model): unnormalised greedy VE results
    alarm = _model("alarm")
    am = alarm.to_markov_model()
    from pgmpy.sampling import BayesianModelSampling

    s = BayesianModelSampling(alarm).forward_sample(size=6, seed=5, show_progress=False)
    r = random.Random(5)
    nodes = sorted(alarm.nodes())
    aq = []
    ve = VariableElimination(am)
    for i in range(6):
        picks = r.sample(nodes, 6)
        qv, ev = picks[:2], {v: str(s.iloc[i][v]) for v in picks[2:]}
        aq.append({"variables": qv, "evidence": ev, "joint": _fac_json(ve.query(qv, ev, show_progress=False))})
    out["alarm_markov"] = {"edges": sorted(sorted(e) for e in am.edges()), "queries": aq}

    # FactorGraph.to_markov_model (FactorGraph.py:303-336) on the 4-cycle potentials
    fg = FactorGraph()
    fg.add_nodes_from(["a", "b", "c", "d"])
    fg.add_factors(*cyc.factors)
    fg.add_nodes_from(cyc.factors)
    fg.add_edges_from([(v, f) for f in cyc.factors for v in f.variables])
    out["factor_graph_to_markov_edges"] = sorted(sorted(e) for e in fg.to_markov_model().edges())
    _dump("markov_cases.json", out)


GENS = {
    "markov": gen_markov,
    "networks": gen_networks,
    "factor_ops": gen_factor_ops,
    "unit_cases": gen_unit_cases,
    "alarm": gen_alarm,
    "alarm_predict": gen_alarm_predict,
    "alarm_bp": gen_alarm_bp,
    "pathfinder_bp": gen_pathfinder_bp,
    "alarm_predict_stochastic": gen_alarm_predict_stochastic,
    "munin_predict": gen_munin_predict,
    "munin_c2": gen_munin_c2,
    "munin_c2_rows": gen_munin_c2_rows,
    "munin_c2_mass": gen_munin_c2_mass,
    "api_extras": gen_api_extras,
}

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--munin-rows", type=int, default=1000)
    a = ap.parse_args()
    _setup()
    for name in (a.only or list(GENS)):
        t0 = time.time()
        if name == "munin_predict":
            gen_munin_predict(a.munin_rows, a.jobs)
        elif name == "munin_c2_rows":
            gen_munin_c2_rows(min(a.jobs, 6))
        elif name == "munin_c2_mass":
            gen_munin_c2_mass(min(a.jobs, 6))
        else:
            GENS[name]()
        print(f"[{name}] {time.time() - t0:.1f}s")
