"""Loaders for the golden fixtures (tests/golden/, written by tests/golden/make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def exists(name):
    return os.path.exists(os.path.join(GOLDEN, name))


def fac_values(fj):
    return np.array([np.inf if v == "inf" else v for v in fj["values"]], dtype=np.float64).reshape(
        [int(c) for c in fj["cardinality"]])


def aligned(values, vars_from, vars_to):
    return np.transpose(values, [list(vars_from).index(v) for v in vars_to]) if len(vars_to) else values


def bn6_network():
    """The 6-node BN of the reference's test_ExactInference.py:22-60 as an oracle ONetwork."""
    from oracle.network import ONetwork

    u = load_json("unit_cases.json")["bn6"]
    nodes = sorted({c["variable"] for c in u["cpds"]})
    states = {c["variable"]: [str(i) for i in range(c["card"])] for c in u["cpds"]}
    parents = {c["variable"]: list(c["evidence"]) for c in u["cpds"]}
    cpts = {c["variable"]: np.array(c["values"]).reshape([c["card"]] + list(c["evidence_card"])) for c in u["cpds"]}
    return ONetwork(nodes, states, parents, cpts)


def munin_predict():
    if not exists("munin_predict.npz"):
        return None
    z = load_npz("munin_predict.npz")
    meta = json.loads(bytes(z["meta"]).decode())
    return {"codes": z["codes"], "map_codes": z["map_codes"], "prob": z["prob"], **meta}


def prob_var_order(columns, candidates, states):
    """Variable order of predict_probability's f"{var}_{state}" columns (state names may hold '_')."""
    order = []
    for c in columns:
        for v in candidates:
            if c.startswith(v + "_") and c[len(v) + 1:] in [str(s) for s in states[v]]:
                if v not in order:
                    order.append(v)
                break
        else:
            raise KeyError(c)
    return order
