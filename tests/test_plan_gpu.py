"""Fused row plans vs the oracle on random networks: components, hidden variables, impossible evidence.

Random BNs (seeded) with zero entries in their CPTs so that some evidence rows
are impossible; for each evidence pattern the batched device plan (fused and
forced-steps executors) must give the oracle's marginals (1e-9 absolute; NaN
exactly where the oracle's 0/0 normalisation gives NaN, DiscreteFactor.py:530),
joint, and MAP (exact when the top-two gap > 1e-9; index 0 on impossible rows,
as np.argmax of an all-NaN joint).
"""
import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


def random_bn(seed, n=14, max_parents=3):
    from oracle.network import ONetwork
    from pgmpy_amd.factors.discrete import TabularCPD
    from pgmpy_amd.models import DiscreteBayesianNetwork

    rng = np.random.default_rng(seed)
    names = [f"v{i:02d}" for i in range(n)]
    card = {v: int(rng.integers(2, 5)) for v in names}
    parents = {}
    for i, v in enumerate(names):
        k = int(rng.integers(0, min(i, max_parents) + 1))
        parents[v] = [names[j] for j in sorted(rng.choice(i, size=k, replace=False))] if k else []
    bn = DiscreteBayesianNetwork()
    bn.add_nodes_from(names)
    bn.add_edges_from([(p, v) for v in names for p in parents[v]])
    cpts = {}
    cpds = []
    for v in names:
        cols = int(np.prod([card[p] for p in parents[v]])) if parents[v] else 1
        t = rng.random((card[v], cols))
        t[rng.random(t.shape) < 0.15] = 0.0
        t[0, t.sum(axis=0) == 0] = 1.0
        t /= t.sum(axis=0, keepdims=True)
        cpts[v] = t.reshape([card[v]] + [card[p] for p in parents[v]])
        sn = {x: [f"s{k}" for k in range(card[x])] for x in [v] + parents[v]}
        cpds.append(TabularCPD(v, card[v], t, parents[v] or None, [card[p] for p in parents[v]] or None,
                               state_names=sn))
    bn.add_cpds(*cpds)
    onet = ONetwork(names, {v: [f"s{k}" for k in range(card[v])] for v in names}, parents, cpts)
    return bn, onet


@pytest.mark.parametrize("seed", range(6))
def test_random_patterns_vs_oracle(gpu, seed):
    from oracle import ve as OVE
    from pgmpy_amd.inference.batch import encode_frame, upload_codes
    from pgmpy_amd.inference.plan import PatternPlan

    bn, onet = random_bn(seed)
    rng = np.random.default_rng(100 + seed)
    names = sorted(bn.nodes())
    for trial in range(4):
        picks = list(rng.choice(names, size=int(rng.integers(3, 9)), replace=False))
        nq = int(rng.integers(1, 4))
        q, e = picks[:nq], picks[nq:]
        n = 40
        rows = {v: [onet.states[v][int(rng.integers(0, onet.card[v]))] for _ in range(n)] for v in e}
        df = pd.DataFrame(rows, columns=e)
        col_of = {c: i for i, c in enumerate(e)}
        codes = upload_codes(encode_frame(bn, df))
        for force in (None, "generic", "steps"):
            plan = PatternPlan(bn, q, e, col_of, force=None if force == "generic" else force)
            if force == "generic":  # table-driven kernel even where the all-affine kernel applies
                from pgmpy_amd import _native as N

                plan.extra_mode = N.ROWS_GENERIC
            out = plan.alloc_outputs(n, marginals=True, joint=True, map_=True)
            plan.run(codes, n, 0, n, out)
            marg, joint, mp = (out["marg"].cpu().numpy(), out["joint"].cpu().numpy(), out["map"].cpu().numpy())
            for r in range(n):
                ev = {v: rows[v][r] for v in e}
                j = OVE.joint(onet, q, ev)
                z = j.sum()
                with np.errstate(invalid="ignore", divide="ignore"):
                    jn = j / z
                np.testing.assert_allclose(joint[:, r], jn.ravel(), atol=1e-12, equal_nan=True)
                exp_m = np.concatenate([jn.sum(axis=tuple(k for k in range(len(q)) if k != i))
                                        for i in range(len(q))])
                np.testing.assert_allclose(marg[:, r], exp_m, atol=1e-12, equal_nan=True)
                if not (z > 0):
                    assert mp[r] == 0
                    continue
                flat = np.sort(jn.ravel())[::-1]
                if flat.size == 1 or (flat[0] - flat[1]) / flat[0] > 1e-9:
                    assert mp[r] == int(np.argmax(jn)), (seed, trial, force, r)


def test_c3_template_factorises_into_components(gpu):
    import random

    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    obs = [v for v in sorted(m.nodes()) if v not in missing]
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    assert plan.kind == "fused"
    d = plan.describe()
    assert d["components"] == 3 and d["evidence_columns"] == 7 and d["values"] == 723


def test_bound_rows_launch_matches_run(gpu):
    """pgm_rows_plan_bind / pgm_rows_bound_run (the prepared launch bench.py times) writes exactly
    what pgm_rows_plan_run writes, re-runs on new codes in place, and validates once at bind."""
    import random

    import torch

    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    rows = 1000
    codes, nodes = forward_sample_codes(m, rows, seed=5)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    ev = np.ascontiguousarray(codes[[pos[v] for v in obs]])
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    d = upload_codes(ev)
    ref = plan.alloc_outputs(rows, marginals=True, map_=True)
    plan.run(d, rows, 0, rows, ref)
    out = plan.alloc_outputs(rows, marginals=True, map_=True)
    bound = plan.bind(d, rows, 0, rows, out)
    bound.run()
    torch.cuda.synchronize()
    assert torch.equal(out["marg"], ref["marg"]) and torch.equal(out["map"], ref["map"])
    d.copy_(upload_codes(np.ascontiguousarray(ev[:, ::-1])))  # new evidence, same buffer
    bound.run()
    plan.run(d, rows, 0, rows, ref)
    torch.cuda.synchronize()
    assert torch.equal(out["marg"], ref["marg"]) and torch.equal(out["map"], ref["map"])
    with pytest.raises(ValueError):
        plan.bind(d, rows, 0, rows, {"marg": torch.empty((plan.n_acc, rows // 2), dtype=torch.float64,
                                                          device=d.device)})


def _munin_template(rows, seed):
    import random

    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    codes, nodes = forward_sample_codes(m, rows, seed=seed)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    ev = np.ascontiguousarray(codes[[pos[v] for v in obs]])
    return PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)}), ev


@pytest.mark.parametrize("rows,n_batches", [(1000, 7), (100_000, 24)])
def test_row_ring_matches_bound_launches(gpu, rows, n_batches):
    """pgm_rows_ring_* (one resident launch consuming posted batches): after a stream of n_batches
    batches over 3 slots (distinct evidence windows, each slot reused), every slot's marginals and MAP
    indices equal the bound one-batch launch on the same rows bit for bit; the ring restarts for a
    second stream; posting past the started count is refused."""
    import torch

    from pgmpy_amd.inference.batch import upload_codes

    plan, ev = _munin_template(rows * 3, seed=17)
    d = upload_codes(ev)
    ld = rows * 3
    slots, refs = [], []
    for s in range(3):
        out = plan.alloc_outputs(rows, marginals=True, map_=True)
        out["marg"].fill_(-1.0)
        slots.append((d, ld, s * rows, out))
        ref = plan.alloc_outputs(rows, marginals=True, map_=True)
        plan.bind(d, ld, s * rows, rows, ref).run()
        refs.append(ref)
    torch.cuda.synchronize()
    err = torch.zeros(1, dtype=torch.int32, device=d.device)
    ring = plan.ring(slots, rows, err=err)
    name, blocks, wg = ring.kernel()
    assert name == "pgm_rows_ring" and blocks >= 256 and wg % 64 == 0
    if n_batches > 3:  # a slot's repeats in one launch: only as a declared replay of unchanged inputs
        with pytest.raises(ValueError, match="replay"):
            ring.run(n_batches)
    for _ in range(2):
        ring.run(n_batches, replay=True)
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        for s in range(3):
            assert torch.equal(slots[s][3]["marg"], refs[s]["marg"]), s
            assert torch.equal(slots[s][3]["map"], refs[s]["map"]), s
        for s in range(3):
            slots[s][3]["marg"].fill_(-1.0)
        torch.cuda.synchronize()
    # started resident first (every workgroup running before the first post), twice: the readiness
    # count carries over launches without a reset
    for _ in range(2):
        ring.start(n_batches, wait_ready=True)
        for b in range(1, n_batches + 1):
            ring.post(b)
        ring.finish()
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        for s in range(3):
            assert torch.equal(slots[s][3]["marg"], refs[s]["marg"]), s
            slots[s][3]["marg"].fill_(-1.0)
        torch.cuda.synchronize()
    ring.start(2)
    ring.post(1)
    with pytest.raises(ValueError):
        ring.post(3)
    with pytest.raises(ValueError):
        ring.finish()  # one batch still unposted
    ring.post(2)
    ring.finish()


@pytest.mark.parametrize("rows,n_shards", [(10_001, 3), (100_000, 2), (7, 4), (1, 1)])
def test_rows_shard_run_matches_run(gpu, rows, n_shards):
    """pgm_rows_shard_run (the C-ABI multi-GPU entry: host rows split into contiguous shards, one
    plan handle + host thread per shard, outputs copied back into the caller's arrays) equals one
    pgm_rows_plan_run over all rows bit for bit — marginals and MAP indices — with the shards on the
    box's GPUs (round robin; several shards share a GPU on a one-GPU box); more shards than rows leave
    empty shards; an out-of-range evidence code raises like run()."""
    import torch

    from pgmpy_amd.inference.batch import download, upload_codes

    plan, ev = _munin_template(rows, seed=23)
    ref = plan.alloc_outputs(rows, marginals=True, map_=True)
    plan.run(upload_codes(ev), rows, 0, rows, ref)
    torch.cuda.synchronize()
    n_dev = torch.cuda.device_count()
    got = plan.shard_run(ev, [i % n_dev for i in range(n_shards)], marginals=True, map_=True)
    assert np.array_equal(got["marg"], download(ref["marg"]), equal_nan=True)
    assert np.array_equal(got["map"], download(ref["map"]))
    only = plan.shard_run(ev, [i % n_dev for i in range(n_shards)], marginals=False, map_=True)
    assert only["marg"] is None and np.array_equal(only["map"], got["map"])
    col = plan.col_of[plan.ev_used[0]]
    bad = ev.copy()
    bad[col, rows // 2] = 200  # not a state of that variable, not the 255 "unobserved" code
    with pytest.raises(IndexError):
        plan.shard_run(bad, [i % n_dev for i in range(n_shards)])


@pytest.mark.parametrize("n_shards", [1, 3])
def test_rows_shard_run_pinned_chunks_against_golden(gpu, n_shards):
    """The persistent, chunk-pipelined pgm_rows_shard_run (r04: per-handle streams and device buffers
    kept from the first call, 256 K-row chunks alternating between two streams, outputs DMA'd into
    pinned host arrays) on the 2,000 reference munin rows tiled to 600,002 rows (so a shard spans
    several chunks and ends on an odd row count): marginals (1e-6 relative) and MAP (exact) against the
    reference fixture, twice in a row through the same handles (the kept buffers are reused)."""
    from pgmpy_amd import _native as N
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from tests.goldens import munin_predict, prob_var_order

    g = munin_predict()
    m = get_example_model("munin")
    observed = list(g["columns"])
    variables = prob_var_order(g["prob_columns"], g["missing"], m.states)
    plan = PatternPlan(m, variables, observed, {v: i for i, v in enumerate(observed)})
    rows = 600_002
    n_ref = g["codes"].shape[1]
    reps = rows // n_ref + 1
    codes = N.HostBuffer((len(observed), rows), np.uint8)
    codes.array[:] = np.tile(g["codes"], (1, reps))[:, :rows]
    out = {"marg": N.HostBuffer((plan.n_acc, rows), np.float64).array,
           "map": N.HostBuffer((rows,), np.int32).array}
    exp = np.tile(g["prob"], (reps, 1))[:rows]
    want = np.tile(g["map_codes"], (reps, 1))[:rows]
    for _ in range(2):
        out["marg"][:] = -1.0
        got = plan.shard_run(codes.array, [0] * n_shards, marginals=True, map_=True, out=out)
        assert got["marg"] is out["marg"]
        np.testing.assert_allclose(got["marg"].T, exp, rtol=1e-6, atol=1e-300)
        idx = got["map"].astype(np.int64)
        digits = {}
        for v, c in reversed(list(zip(variables, plan.cards))):
            digits[v] = idx % c
            idx //= c
        np.testing.assert_array_equal(np.stack([digits[v] for v in g["missing"]], axis=1), want)


def test_row_ring_exits_without_posts(gpu):
    """Every exit path of the resident kernel ends the launch: cancel() with batches never posted,
    and the timeout (the waves give up waiting; finish() then reports the timeout)."""
    import time

    import torch

    from pgmpy_amd.inference.batch import upload_codes

    rows = 2000
    plan, ev = _munin_template(rows, seed=3)
    d = upload_codes(ev)
    out = plan.alloc_outputs(rows, marginals=True)
    ring = plan.ring([(d, rows, 0, out)], rows)
    t0 = time.perf_counter()
    ring.start(4, timeout_s=5.0)
    ring.post(1)
    ring.cancel()  # three batches never posted
    assert time.perf_counter() - t0 < 4.0
    ring.start(3, timeout_s=0.05)
    time.sleep(0.3)  # past the deadline: every wave waiting for batch 0 has left
    ring.post(3)
    with pytest.raises(RuntimeError, match="timed out"):
        ring.finish()
    ring.run(3, replay=True)  # usable again
    torch.cuda.synchronize()
    ref = plan.alloc_outputs(rows, marginals=True)
    plan.bind(d, rows, 0, rows, ref).run()
    torch.cuda.synchronize()
    assert torch.equal(out["marg"], ref["marg"])
    with pytest.raises(ValueError):  # odd row counts break the two-rows-per-lane contract
        plan.ring([(d, rows, 0, plan.alloc_outputs(rows - 1, marginals=True))], rows - 1)


@pytest.mark.parametrize("rows", [1000, 100_000, 1_000_000])
def test_direct_queue_launch_matches_bound(gpu, rows):
    """pgm_dq_bind_rows / pgm_dq_launch (the AQL-packet launch of the same specialised kernel on a
    user-mode HSA queue) writes bit-for-bit what the HIP-launched bound run writes, including after
    many back-to-back dispatches (the completion-signal ring wraps) and on new codes in place; the
    queue timer reports a positive GPU span."""
    import random

    import torch

    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import DirectQueue, PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    codes, nodes = forward_sample_codes(m, rows, seed=11)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    ev = np.ascontiguousarray(codes[[pos[v] for v in obs]])
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    d = upload_codes(ev)
    ref = plan.alloc_outputs(rows, marginals=True, map_=True)
    plan.bind(d, rows, 0, rows, ref).run()
    torch.cuda.synchronize()
    out = plan.alloc_outputs(rows, marginals=True, map_=True)
    q = DirectQueue()
    direct = plan.bind(d, rows, 0, rows, out).direct(q)
    q.timer_start()
    for _ in range(300):  # > the 256-signal ring
        direct.run()
    ms = q.timer_stop_ms()
    q.sync()
    assert ms > 0.0
    assert torch.equal(out["marg"], ref["marg"]) and torch.equal(out["map"], ref["map"])
    d.copy_(upload_codes(np.ascontiguousarray(ev[:, ::-1])))  # new evidence in the same buffer
    torch.cuda.synchronize()
    out["marg"].zero_()
    torch.cuda.synchronize()
    direct.run()
    direct.sync()
    plan.bind(d, rows, 0, rows, ref).run()
    torch.cuda.synchronize()
    assert torch.equal(out["marg"], ref["marg"]) and torch.equal(out["map"], ref["map"])
    # HIP writes the inputs and clears the outputs with NO synchronize before the next direct launch: the
    # first dispatch after a sync drains HIP work itself; the launch releases at system scope
    # on its own completion (pgm_dq_launch_release), so a wait suffices before HIP reads the outputs
    d.copy_(upload_codes(ev))
    out["marg"].zero_()
    out["map"].zero_()
    direct.run_release()
    q.wait()
    plan.bind(d, rows, 0, rows, ref).run()
    torch.cuda.synchronize()
    assert torch.equal(out["marg"], ref["marg"]) and torch.equal(out["map"], ref["map"])
    direct.run()  # the dispatch after a released launch acquires again (as after a sync)
    q.sync()


def test_direct_group_launch_matches_bound(gpu):
    """pgm_dq_launch_group (independent row batches dispatched with only the first packet carrying
    the barrier bit): after many groups every batch's output equals its own HIP-launched bound run
    bit for bit, the timer spans the group, sync waits for all members; a group that repeats a
    launch or shares an output buffer is refused."""
    import random

    import torch

    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import DirectGroup, DirectQueue, PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    rows, nb = 100_000, 4
    codes, nodes = forward_sample_codes(m, rows * nb, seed=21)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    ev = np.ascontiguousarray(codes[[pos[v] for v in obs]])
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    d = upload_codes(ev)
    refs, outs, bounds = [], [], []
    for i in range(nb):
        ref = plan.alloc_outputs(rows, marginals=True, map_=True)
        plan.bind(d, rows * nb, i * rows, rows, ref).run()
        refs.append(ref)
        out = plan.alloc_outputs(rows, marginals=True, map_=True)
        outs.append(out)
        bounds.append(plan.bind(d, rows * nb, i * rows, rows, out))
    torch.cuda.synchronize()
    q = DirectQueue()
    rs = [b.direct(q) for b in bounds]
    grp = DirectGroup(rs)
    q.timer_start()
    for _ in range(100):  # 400 dispatches: the signal ring wraps mid-group
        grp.run()
    ms = q.timer_stop_ms()
    q.sync()
    assert ms > 0.0
    for out, ref in zip(outs, refs):
        assert torch.equal(out["marg"], ref["marg"]) and torch.equal(out["map"], ref["map"])
    for o in outs:
        o["marg"].zero_()
    torch.cuda.synchronize()
    grp.run()
    q.sync()
    for out, ref in zip(outs, refs):
        assert torch.equal(out["marg"], ref["marg"])
    with pytest.raises(ValueError):
        DirectGroup([rs[0], rs[0]])
    with pytest.raises(ValueError):
        DirectGroup([rs[0], plan.bind(d, rows * nb, rows, rows, outs[0]).direct(q)])
    # distinct base pointers, overlapping bytes (views of one buffer): refused too
    m = plan.n_acc * rows
    flat = torch.empty(3 * m, dtype=torch.float64, device=d.device)
    va = {"marg": flat[:m].view(plan.n_acc, rows)}
    vb = {"marg": flat[m // 2:m // 2 + m].view(plan.n_acc, rows)}
    ra = plan.bind(d, rows * nb, 0, rows, va).direct(q)
    rb = plan.bind(d, rows * nb, rows, rows, vb).direct(q)
    with pytest.raises(ValueError, match="overlapping"):
        DirectGroup([ra, rb])
    vc = {"marg": flat[m:2 * m].view(plan.n_acc, rows)}  # adjacent, not overlapping: accepted
    DirectGroup([ra, plan.bind(d, rows * nb, rows, rows, vc).direct(q)])


def test_direct_queues_in_parallel(gpu):
    """Independent row batches on separate user-mode queues (bench.py --queues): every batch's
    output equals its HIP-launched bound run after interleaved dispatches; the joined tick spans of
    the queues are ordered and share one clock."""
    import random

    import torch

    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import DirectQueue, PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    rows, nq = 50_000, 3
    codes, nodes = forward_sample_codes(m, rows * nq, seed=23)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    ev = np.ascontiguousarray(codes[[pos[v] for v in obs]])
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    d = upload_codes(ev)
    qs = [DirectQueue() for _ in range(nq)]
    refs, outs, rs = [], [], []
    for i in range(nq):
        ref = plan.alloc_outputs(rows, marginals=True, map_=True)
        plan.bind(d, rows * nq, i * rows, rows, ref).run()
        refs.append(ref)
        out = plan.alloc_outputs(rows, marginals=True, map_=True)
        outs.append(out)
        rs.append(plan.bind(d, rows * nq, i * rows, rows, out).direct(qs[i]))
    torch.cuda.synchronize()
    for q in qs:
        q.timer_start()
    for _ in range(50):
        for r in rs:
            r.run()
    spans = [q.timer_stop_ticks() for q in qs]
    for q in qs:
        q.sync()
    assert all(b > a > 0 for a, b, _ in spans) and len({f for _, _, f in spans}) == 1
    for out, ref in zip(outs, refs):
        assert torch.equal(out["marg"], ref["marg"]) and torch.equal(out["map"], ref["map"])


def test_dispatch_floor_kernel(gpu):
    """PGM_ROWS_FLOOR (bench.py's dispatch floor): the floor kernel writes every marginal row with the
    sum of the plan's distinct evidence codes of that row (the loads and stores the specialised kernel
    makes, no CPT arithmetic), over both launchers; plans without the specialised kernel refuse it."""
    import random

    import torch

    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import DirectQueue, PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    rows = 5000
    codes, nodes = forward_sample_codes(m, rows, seed=13)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    ev = np.ascontiguousarray(codes[[pos[v] for v in obs]])
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    d = upload_codes(ev)
    cols = [plan.col_of[v] for v in plan.ev_used]
    expect = ev[cols].astype(np.float64).sum(axis=0)
    for direct in (False, True):
        out = plan.alloc_outputs(rows, marginals=True)
        b = plan.bind(d, rows, 0, rows, out, floor=True)
        if direct:
            q = DirectQueue()
            r = b.direct(q)
            r.run()
            q.sync()
        else:
            b.run()
        torch.cuda.synchronize()
        got = out["marg"].cpu().numpy()
        for k in range(plan.n_acc):
            np.testing.assert_array_equal(got[k], expect)


def test_direct_queue_needs_specialised_kernel(gpu):
    """A bound launch that runs an AOT kernel (no hipRTC code object) cannot be re-bound to the
    direct queue: ValueError, nothing dispatched."""
    import random

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    codes, nodes = forward_sample_codes(m, 256, seed=12)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    plan.extra_mode = N.ROWS_GENERIC
    d = upload_codes(np.ascontiguousarray(codes[[pos[v] for v in obs]]))
    bound = plan.bind(d, 256, 0, 256, plan.alloc_outputs(256, marginals=True))
    with pytest.raises(ValueError):
        bound.direct()


@pytest.mark.parametrize("seed", range(6))
def test_specialised_kernel_bit_identical(gpu, seed):
    """The plan-specialised (hipRTC) row kernel agrees with the AOT kernels (k_rows_affine and the
    table-driven k_rows) to the last place: marginals, MAP index (where the top-two gap is not a
    tie) and MAP gap, NaN rows of impossible evidence, and the out-of-range evidence flag."""
    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference.batch import encode_frame, upload_codes
    from pgmpy_amd.inference.plan import PatternPlan

    bn, onet = random_bn(seed)
    rng = np.random.default_rng(500 + seed)
    names = sorted(bn.nodes())
    checked = 0
    for trial in range(60):
        if checked >= 4:
            break
        picks = list(rng.choice(names, size=int(rng.integers(6, 13)), replace=False))
        nq = int(rng.integers(1, 3))
        q, e = picks[:nq], picks[nq:]
        n = 300 if seed % 2 == 0 else 301
        rows = {v: [onet.states[v][int(rng.integers(0, onet.card[v]))] for _ in range(n)] for v in e}
        df = pd.DataFrame(rows, columns=e)
        col_of = {c: i for i, c in enumerate(e)}
        codes = upload_codes(encode_frame(bn, df))
        plan = PatternPlan(bn, q, e, col_of)
        if plan.kind != "fused" or plan.kernel_name() != "pgm_rows_jit":
            continue
        outs = {}
        for name, extra in (("jit", 0), ("aot", N.ROWS_NO_JIT), ("generic", N.ROWS_GENERIC)):
            plan.extra_mode = extra
            o = plan.alloc_outputs(n, marginals=True, map_=True, gap=True)
            err = torch.zeros(1, dtype=torch.int32, device=codes.device)
            plan.run(codes, n, 0, n, o, err=err)
            outs[name] = (o, int(err.item()))
        plan.extra_mode = 0
        for name in ("aot", "generic"):
            a, b = outs["jit"][0], outs[name][0]
            assert torch.equal(a["marg"].isnan(), b["marg"].isnan())
            # same arithmetic order as k_rows_affine (bit-identical there); the table-driven k_rows
            # may round differently in the last place
            torch.testing.assert_close(a["marg"], b["marg"], rtol=1e-14, atol=0, equal_nan=True)
            torch.testing.assert_close(a["gap"], b["gap"], rtol=1e-12, atol=1e-15)
            clear = a["gap"] > 1e-9
            assert torch.equal(a["map"][clear], b["map"][clear]), name
            assert outs["jit"][1] == outs[name][1] == 0
        # an out-of-range code raises the flag and reads state 0 in both kernels
        used = [col_of[v] for v in plan.ev_used]
        if used:
            bad = codes.clone()
            bad[used[0], :7] = 250
            for extra in (0, N.ROWS_NO_JIT):
                plan.extra_mode = extra
                o = plan.alloc_outputs(n, marginals=True)
                err = torch.zeros(1, dtype=torch.int32, device=codes.device)
                plan.run(bad, n, 0, n, o, err=err)
                assert int(err.item()) == 1
            plan.extra_mode = 0
        checked += 1
    assert checked >= 1


@pytest.mark.parametrize("rows", [100_000, 100_001, 400_000, 400_001])
def test_specialised_kernel_large_batches(gpu, rows):
    """Large batches (>= 50k rows): even row counts take the two-rows-per-thread specialised kernel
    (16-B stores, 2-byte code loads), odd ones the one-row kernel; both bit-identical to k_rows_affine.
    The bound launch reports which one it runs (pgm_rows_bound_kernel)."""
    import random

    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    codes, nodes = forward_sample_codes(m, 2000, seed=11)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    ev = np.ascontiguousarray(np.tile(codes[[pos[v] for v in obs]], (1, rows // 2000 + 1))[:, :rows])
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    d = upload_codes(ev)
    res = []
    for extra in (0, N.ROWS_NO_JIT):
        plan.extra_mode = extra
        o = plan.alloc_outputs(rows, marginals=True, map_=True, gap=True)
        plan.run(d, rows, 0, rows, o)
        res.append(o)
    plan.extra_mode = 0
    torch.cuda.synchronize()
    for k in ("marg", "map", "gap"):
        assert torch.equal(res[0][k], res[1][k]), k
    o = plan.alloc_outputs(rows, marginals=True)
    name, blocks, wg = plan.bind(d, rows, 0, rows, o).kernel()
    per_block = wg * (2 if rows % 2 == 0 else 1)
    assert name == ("pgm_rows_jit2" if rows % 2 == 0 else "pgm_rows_jit")
    assert blocks == (rows + per_block - 1) // per_block


@pytest.mark.parametrize("row0,n", [(0, 1), (37, 1), (5, 255), (1000, 257), (2, 100_000), (3, 100_000), (2, 400_000),
                                   (3, 400_000)])
def test_specialised_kernel_row_windows(gpu, row0, n):
    """Rows [row0, row0 + n) of a wider code matrix (ld > n): single rows, ragged counts, odd and even
    offsets (the two-rows kernel needs an even row0) give what a contiguous copy of the window gives."""
    import random

    import torch

    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    codes, nodes = forward_sample_codes(m, 3000, seed=21)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    ld = row0 + n + 3
    ev = np.ascontiguousarray(np.tile(codes[[pos[v] for v in obs]], (1, ld // 3000 + 1))[:, :ld])
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    full = upload_codes(ev)
    win = upload_codes(np.ascontiguousarray(ev[:, row0:row0 + n]))
    a = plan.alloc_outputs(n, marginals=True, map_=True)
    b = plan.alloc_outputs(n, marginals=True, map_=True)
    plan.run(full, ld, row0, n, a)
    plan.run(win, n, 0, n, b)
    torch.cuda.synchronize()
    assert torch.equal(a["marg"], b["marg"]) and torch.equal(a["map"], b["map"])
