"""Primitive-kernel parity on the GPU: pgm_contract / pgm_gather / pgm_argmax / pgm_rows_*.

Each kernel is checked against the numpy arithmetic the reference itself runs
(np.einsum / np.max / np.argmax / basic indexing: DiscreteFactor.py:408,480,614,
771-777; compat_fns.py:53-74).  Tolerance: 1e-12 relative for sums (fp64,
different summation order), exact for copies, max and argmax.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _e():
    from pgmpy_amd import engine

    return engine


@pytest.mark.parametrize("seed", range(12))
def test_contract_random_einsum(gpu, seed):
    E = _e()
    rng = np.random.default_rng(seed)
    labels = list("abcdefg")
    card = {l: int(rng.integers(1, 6)) for l in labels}
    la = list(rng.choice(labels, size=int(rng.integers(1, 5)), replace=False))
    lb = list(rng.choice(labels, size=int(rng.integers(1, 5)), replace=False))
    a = rng.random([card[l] for l in la])
    b = rng.random([card[l] for l in lb])
    union = list(dict.fromkeys(la + lb))
    keep = [l for l in union if rng.random() < 0.6]
    rng.shuffle(keep)
    A, B = E.to_device(a), E.to_device(b)
    ref = np.einsum(a, [labels.index(l) for l in la], b, [labels.index(l) for l in lb],
                    [labels.index(l) for l in keep])
    got = E.to_host(E.contract(A, la, B, lb, keep, reduce="sum", combine="mul"))
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=0)
    # max-product
    full = np.einsum(a, [labels.index(l) for l in la], b, [labels.index(l) for l in lb],
                     [labels.index(l) for l in union])
    red = tuple(i for i, l in enumerate(union) if l not in keep)
    refm = np.max(full, axis=red) if red else full
    refm = np.transpose(refm, [[l for l in union if l in keep].index(l) for l in keep]) if keep else refm
    gotm = E.to_host(E.contract(A, la, B, lb, keep, reduce="max", combine="mul"))
    np.testing.assert_array_equal(gotm, refm)


def test_contract_large_reduction_split(gpu):
    """Tiny output, huge reduction -> split-K path with the finalize kernel."""
    E = _e()
    rng = np.random.default_rng(1)
    a = rng.random((3, 1 << 20))
    A = E.to_device(a)
    got = E.to_host(E.contract(A, ["x", "y"], None, None, ["x"], reduce="sum", combine="copy"))
    np.testing.assert_allclose(got, a.sum(axis=1), rtol=1e-12)
    got0 = E.to_host(E.contract(A, ["x", "y"], None, None, ["y"], reduce="sum", combine="copy"))
    np.testing.assert_allclose(got0, a.sum(axis=0), rtol=1e-12)
    tot = E.to_host(E.total(A))
    np.testing.assert_allclose(tot, a.sum(), rtol=1e-12)
    mx = E.to_host(E.contract(A, ["x", "y"], None, None, ["x"], reduce="max", combine="copy"))
    np.testing.assert_array_equal(mx, a.max(axis=1))


def test_divide_and_normalize_semantics(gpu):
    E = _e()
    a = np.array([[0.0, 1.0], [2.0, 0.0]])
    b = np.array([0.0, 2.0])
    A, B = E.to_device(a), E.to_device(b)
    got = E.to_host(E.contract(A, ["x1", "x2"], B, ["x1"], ["x1", "x2"], combine="div"))
    # DiscreteFactor.py:859-863: 0/0 -> 0, x/0 -> inf
    np.testing.assert_array_equal(got, np.array([[0.0, np.inf], [1.0, 0.0]]))
    z = E.to_device(np.zeros(4))
    E.normalize_(z)
    assert np.isnan(E.to_host(z)).all()


def test_argmax_first_index_and_nan(gpu):
    E = _e()
    x = np.array([[1.0, 3.0, 3.0, 2.0], [0.0, 0.0, 0.0, 0.0], [1.0, np.nan, 5.0, np.nan]])
    X = E.to_device(x)
    got = E.to_host(E.argmax_rows(X, ["r", "i"], row_label="r").double()).astype(int)
    assert list(got) == [int(np.argmax(r)) for r in x]


def test_gather_per_row(gpu):
    import torch

    E = _e()
    rng = np.random.default_rng(5)
    a = rng.random((3, 4, 5))
    n = 1000
    codes = np.stack([rng.integers(0, 4, n), rng.integers(0, 5, n)]).astype(np.uint8)
    C = torch.from_numpy(codes).to(gpu)
    A = E.to_device(a)
    out = E.gather(A, ["x", "y", "z"], {"y": (None, 0), "z": (None, 1)}, ["x", E.ROW], codes=C, ld=n, n_rows=n)
    got = E.to_host(out)
    ref = np.stack([a[:, codes[0, r], codes[1, r]] for r in range(n)], axis=1)
    np.testing.assert_array_equal(got, ref)
    bad = torch.from_numpy(np.full((2, n), 7, dtype=np.uint8)).to(gpu)
    with pytest.raises(IndexError):
        E.gather(A, ["x", "y", "z"], {"y": (None, 0), "z": (None, 1)}, ["x", E.ROW], codes=bad, ld=n, n_rows=n)


def test_rows_plan_matches_numpy(gpu):
    """Hand-built fused plan: 2 query dims, 1 hidden dim, 3 factors with evidence."""
    import ctypes

    import torch

    from pgmpy_amd import _native as N

    rng = np.random.default_rng(11)
    cq0, cq1, ch, ce0, ce1 = 3, 4, 2, 5, 3
    f0 = rng.random((cq0, ce0))            # (q0, e0)
    f1 = rng.random((cq1, cq0, ch))        # (q1, q0, h)
    f2 = rng.random((ch, ce1, cq1))        # (h, e1, q1)
    vals = np.concatenate([f0.ravel(), f1.ravel(), f2.ravel()])
    P = N.RowsPlan()
    P.n_loop, P.n_query, P.n_fac, P.n_ev, P.n_values = 3, 2, 3, 2, vals.size
    P.n_comp, P.n_marg, P.n_joint = 1, cq0 + cq1, cq0 * cq1
    P.comp_loop_begin[0], P.comp_n_query[0], P.comp_loop_end[0] = 0, 2, 3
    P.comp_fac_begin[0], P.comp_fac_end[0] = 0, 3
    for i, c in enumerate([cq0, cq1, ch]):
        P.loop_card[i] = c
    P.loop_marg_off[0], P.loop_marg_off[1], P.loop_marg_off[2] = 0, cq0, -1
    P.loop_map_stride[0], P.loop_map_stride[1] = cq1, 1
    P.fac_base[0], P.fac_base[1], P.fac_base[2] = 0, f0.size, f0.size + f1.size
    s0, s1, s2 = [x // 8 for x in f0.strides], [x // 8 for x in f1.strides], [x // 8 for x in f2.strides]
    # loop dims: 0=q0, 1=q1, 2=h
    P.fac_stride[0][0] = s0[0]
    P.fac_stride[1][1], P.fac_stride[1][0], P.fac_stride[1][2] = s1[0], s1[1], s1[2]
    P.fac_stride[2][2], P.fac_stride[2][1] = s2[0], s2[2]
    P.fac_ev_begin[0], P.fac_ev_end[0] = 0, 1
    P.fac_ev_begin[1], P.fac_ev_end[1] = 1, 1
    P.fac_ev_begin[2], P.fac_ev_end[2] = 1, 2
    P.ev_col[0], P.ev_stride[0], P.ev_card[0] = 0, s0[1], ce0
    P.ev_col[1], P.ev_stride[1], P.ev_card[1] = 1, s2[1], ce1
    L = N.lib()
    h = ctypes.c_void_p()
    N.check(L.pgm_rows_plan_create(ctypes.byref(P), vals.ctypes.data_as(ctypes.c_void_p), ctypes.byref(h)))
    n = 777
    codes = np.stack([rng.integers(0, ce0, n), rng.integers(0, ce1, n)]).astype(np.uint8)
    C = torch.from_numpy(codes).to(gpu)
    marg = torch.empty((cq0 + cq1, n), dtype=torch.float64, device=gpu)
    joint = torch.empty((cq0 * cq1, n), dtype=torch.float64, device=gpu)
    mp = torch.empty(n, dtype=torch.int32, device=gpu)
    gap = torch.empty(n, dtype=torch.float64, device=gpu)
    err = torch.zeros(1, dtype=torch.int32, device=gpu)
    mode = N.ROWS_MARGINALS | N.ROWS_JOINT | N.ROWS_MAP | N.ROWS_MAPGAP
    N.check(L.pgm_rows_plan_run(h, mode, N.ptr(C), n, 0, n, N.ptr(marg), N.ptr(joint), n, N.ptr(mp), N.ptr(gap),
                                N.ptr(err), N.stream_handle()))
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    joint_h, marg_h, mp_h = joint.cpu().numpy(), marg.cpu().numpy(), mp.cpu().numpy()
    for r in range(n):
        e0, e1 = codes[0, r], codes[1, r]
        j = np.einsum("a,bah,hb->ab", f0[:, e0], f1, f2[:, e1, :])
        z = j.sum()
        np.testing.assert_allclose(joint_h[:, r], (j / z).ravel(), rtol=1e-12)
        np.testing.assert_allclose(marg_h[:cq0, r], j.sum(1) / z, rtol=1e-12)
        np.testing.assert_allclose(marg_h[cq0:, r], j.sum(0) / z, rtol=1e-12)
        assert int(mp_h[r]) == int(np.argmax(j))
    N.check(L.pgm_rows_plan_destroy(h))


@pytest.mark.parametrize("seed", range(10))
def test_contract_row_mode_shapes(gpu, seed):
    """Shapes that take the row-mode kernel (innermost output dim >= 64), with and without
    reductions, transposed operands, broadcast operands and split reductions."""
    E = _e()
    rng = np.random.default_rng(1000 + seed)
    labels = list("abcdef")
    card = {l: int(rng.integers(2, 6)) for l in labels}
    card["r"] = int(rng.choice([64, 100, 257, 1000]))  # row-like axis
    la = list(rng.choice(labels, size=int(rng.integers(1, 4)), replace=False)) + ["r"]
    lb = list(rng.choice(labels, size=int(rng.integers(0, 3)), replace=False))
    if seed % 2:
        lb = lb + ["r"]
    rng.shuffle(la)
    a = rng.random([card[l] for l in la])
    b = rng.random([card[l] for l in lb]) if lb else np.array(rng.random())
    union = list(dict.fromkeys(la + lb))
    keep = [l for l in union if l != "r" and rng.random() < 0.5] + ["r"]
    A, B = E.to_device(a), E.to_device(b)
    idx = {l: i for i, l in enumerate(union)}
    ref = np.einsum(a, [idx[l] for l in la], b, [idx[l] for l in lb], [idx[l] for l in keep])
    got = E.to_host(E.contract(A, la, B, lb, keep, reduce="sum", combine="mul"))
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-300)
    full = np.einsum(a, [idx[l] for l in la], b, [idx[l] for l in lb], list(range(len(union))))
    red = tuple(i for i, l in enumerate(union) if l not in keep)
    refm = np.max(full, axis=red) if red else full
    refm = np.transpose(refm, [[l for l in union if l in keep].index(l) for l in keep])
    np.testing.assert_array_equal(E.to_host(E.contract(A, la, B, lb, keep, reduce="max", combine="mul")), refm)
    # elementwise divide with a broadcast operand over the row axis
    keep2 = union
    D = E.contract(A, la, B, lb, keep2, combine="div")
    with np.errstate(divide="ignore", invalid="ignore"):
        refd = np.einsum(a, [idx[l] for l in la], list(range(len(union)))) if False else None
    bb = np.broadcast_to(np.einsum(b, [idx[l] for l in lb], sorted(idx[l] for l in lb)).reshape(
        [card[l] if l in lb else 1 for l in union]), [card[l] for l in union]) if lb else b
    aa = np.broadcast_to(np.einsum(a, [idx[l] for l in la], sorted(idx[l] for l in la)).reshape(
        [card[l] if l in la else 1 for l in union]), [card[l] for l in union])
    with np.errstate(divide="ignore", invalid="ignore"):
        q = aa / bb
    q[np.isnan(q)] = 0
    np.testing.assert_allclose(E.to_host(D), q, rtol=1e-15)


def test_contract_row_mode_split_reduction(gpu):
    """Few outputs along a 512-wide row axis, long reduction: row mode + split-K + finalize."""
    E = _e()
    rng = np.random.default_rng(7)
    a = rng.random((4000, 512))
    b = rng.random((4000,))
    A, B = E.to_device(a), E.to_device(b)
    got = E.to_host(E.contract(A, ["k", "r"], B, ["k"], ["r"], reduce="sum", combine="mul"))
    np.testing.assert_allclose(got, b @ a, rtol=1e-12)


def test_product_n_and_graph_replay(gpu):
    """pgm_product_n (up to 8 broadcast operands, row and flat mode) and HIP-graph replay."""
    import torch

    from pgmpy_amd.program import Program

    E = _e()
    rng = np.random.default_rng(3)
    for rows in (1, 300):
        a = rng.random((3, 4, rows))
        b = rng.random((4, rows))
        c = rng.random((3,))
        d = rng.random((5, 3, rows))
        ops = [(E.to_device(a), ["x", "y", "r"]), (E.to_device(b), ["y", "r"]), (E.to_device(c), ["x"]),
               (E.to_device(d), ["z", "x", "r"])]
        got = E.to_host(E.product_n(ops, ["z", "x", "y", "r"]))
        ref = np.einsum("xyr,yr,x,zxr->zxyr", a, b, c, d)
        np.testing.assert_allclose(got, ref, rtol=1e-15)
    # ratio pair: C = X * (N / D) with 0/0 -> 0 (x/0 -> inf)
    X = rng.random((3, 50))
    Nn = rng.random((3, 50))
    Dd = rng.random((3, 50))
    Nn[0, :5] = 0.0
    Dd[0, :5] = 0.0
    Dd[1, :3] = 0.0
    from pgmpy_amd import _native as NN

    got = E.to_host(E.product_n([(E.to_device(X), ["a", "r"]), (E.to_device(Nn), ["a", "r"]),
                                 (E.to_device(Dd), ["a", "r"])], ["a", "r"],
                                kinds=[NN.PRODN_MUL, NN.PRODN_RATIO, NN.PRODN_DEN]))
    with np.errstate(divide="ignore", invalid="ignore"):
        r = Nn / Dd
    r[np.isnan(r)] = 0
    np.testing.assert_array_equal(got, X * r)
    # a captured program: out = (A*B) summed over y, replayed after A changes in place
    A = E.to_device(rng.random((6, 500)))
    B = E.to_device(rng.random((6,)))
    prog = Program()
    out = prog.contract(A, ["y", "r"], B, ["y"], ["r"], reduce="sum", combine="mul")
    prog.capture()
    prog.run()
    torch.cuda.synchronize()
    np.testing.assert_allclose(E.to_host(out), E.to_host(B) @ E.to_host(A), rtol=1e-12)
    A.mul_(2.0)
    prog.run()
    torch.cuda.synchronize()
    np.testing.assert_allclose(E.to_host(out), E.to_host(B) @ E.to_host(A), rtol=1e-12)


@pytest.mark.parametrize("shape", [
    # (batch labels, M labels, N labels, K labels) as {label: card}
    ({}, {"m": 3000}, {"n": 120}, {"k": 112}),
    ({"b": 5}, {"m": 70}, {"n": 33}, {"k": 17}),
    ({"b": 3, "c": 2}, {"m1": 9, "m2": 7}, {"n1": 5, "n2": 13}, {"k1": 4, "k2": 6}),
    ({}, {"m": 16}, {"n": 16}, {"k": 8}),
    ({}, {"m": 65}, {"n": 129}, {"k": 700}),
    # the 16 x 128 tile (M <= 16) and the 128 x 64 tile (64 < M <= 128), ragged edges, table groups
    ({"b": 4}, {"m": 16}, {"n": 300}, {"k": 37}),
    ({"b": 2}, {"m1": 10, "m2": 10}, {"n": 200}, {"k1": 5, "k2": 25}),
    # more than 65,535 batch entries: the batch continues in grid.z
    ({"b1": 300, "b2": 250}, {"m": 16}, {"n": 16}, {"k": 8}),
])
def test_pair_gemm_matches_einsum(gpu, shape):
    """FP64 MFMA dense steps (pgm_gemm) vs numpy, with permuted / non-contiguous operands."""
    from pgmpy_amd import engine as E

    rng = np.random.default_rng(11)
    bt, mm, nn, kk = shape
    card = {**bt, **mm, **nn, **kk}
    la = list(mm) + list(kk) + list(bt)
    lb = list(kk)[::-1] + list(bt) + list(nn)
    rng.shuffle(la)
    rng.shuffle(lb)
    A = rng.random([card[l] for l in la])
    B = rng.random([card[l] for l in lb])
    keep = list(bt) + list(mm) + list(nn)
    C = E.pair_gemm(E.to_device(A), la, E.to_device(B), lb, keep, force=True)
    assert C is not None
    labels = keep
    sym = {l: i for i, l in enumerate(card)}
    ref = np.einsum(A, [sym[l] for l in la], B, [sym[l] for l in lb], [sym[l] for l in labels])
    np.testing.assert_allclose(E.to_host(C), ref, rtol=1e-12, atol=1e-12)
    # a transposed view of A and an output in another label order: addressed through the tables
    At = E.to_device(A).permute(*reversed(range(A.ndim)))
    keep2 = keep[::-1]
    C2 = E.pair_gemm(At, la[::-1], E.to_device(B), lb, keep2, force=True)
    np.testing.assert_allclose(E.to_host(C2), E.to_host(E.contract(C, labels, None, None, keep2, combine="copy")),
                               rtol=1e-12, atol=1e-12)


def test_pair_gemm_unit_stride_lane_orders(gpu):
    """pgm_gemm tile loads follow each operand's unit-stride axis: A stored m-innermost (m-fast
    lanes), B stored k-innermost (k-fast lanes), ragged tile edges, a batch group."""
    from pgmpy_amd import engine as E

    rng = np.random.default_rng(12)
    A = rng.random((3, 37, 100))  # [b, k, m]
    B = rng.random((3, 70, 37))   # [b, n, k]
    C = E.pair_gemm(E.to_device(A), ["b", "k", "m"], E.to_device(B), ["b", "n", "k"], ["b", "m", "n"], force=True)
    assert C is not None
    ref = np.einsum("bkm,bnk->bmn", A, B)
    np.testing.assert_allclose(E.to_host(C), ref, rtol=1e-12, atol=1e-12)


def test_pair_gemm_declines_non_gemm_steps(gpu):
    from pgmpy_amd import engine as E

    A = E.to_device(np.ones((4, 5)))
    B = E.to_device(np.ones((5, 3)))
    assert E.pair_gemm(A, ["a", "k"], B, ["k", "b"], ["a", "b"]) is None  # too small
    A = E.to_device(np.ones((64, 64, 2)))
    B = E.to_device(np.ones((64, 64)))
    assert E.pair_gemm(A, ["a", "k", "p"], B, ["k", "b"], ["a", "b"]) is None  # p summed out of A alone


def test_contract_factors_gemm_steps_match_numpy(gpu):
    """A chain whose greedy steps mix GEMM-shaped and generic contractions."""
    from pgmpy_amd import engine as E
    from pgmpy_amd.inference.contraction import contract_factors

    rng = np.random.default_rng(5)
    card = {"a": 40, "b": 24, "c": 30, "d": 3, "e": 50}
    specs = [["a", "b"], ["b", "c", "d"], ["c", "e"], ["d"], ["e", "a"]]
    arrs = [rng.random([card[l] for l in ls]) for ls in specs]
    got = E.to_host(contract_factors([(E.to_device(x), ls) for x, ls in zip(arrs, specs)], ["a", "d"]))
    sym = {l: i for i, l in enumerate(card)}
    args = []
    for x, ls in zip(arrs, specs):
        args += [x, [sym[l] for l in ls]]
    ref = np.einsum(*args, [sym["a"], sym["d"]])
    np.testing.assert_allclose(got, ref, rtol=1e-12)


def test_program_batch_matches_eager(gpu):
    """Independent small contractions and gathers recorded in one batch (pgm_batch_*: one launch)
    give the same results as individual launches, replayed directly and from a HIP graph."""
    import ctypes

    from pgmpy_amd import _native as N
    from pgmpy_amd import engine as E
    from pgmpy_amd.program import Program

    rng = np.random.default_rng(3)
    jobs = [
        (rng.random((3, 4, 5)), ["a", "b", "c"], rng.random((5, 6)), ["c", "d"], ["a", "d"], "sum", "mul"),
        (rng.random((7, 2)), ["x", "y"], None, None, ["y"], "max", "copy"),
        (rng.random((4, 9)), ["p", "q"], rng.random((9,)) + 0.5, ["q"], ["p", "q"], None, "div"),
        (rng.random((2, 3, 4)), ["u", "v", "w"], None, None, ["w", "u", "v"], None, "copy"),
        (rng.random((300, 40)), ["m", "k"], rng.random((40, 50)), ["k", "n"], ["m", "n"], "sum", "mul"),
        (rng.random((6,)), ["s"], rng.random((5,)), ["t"], ["t", "s"], None, "add"),
        # rows innermost and even: the 16-B output-pair form (separator marginal, max-product message)
        (rng.random((4, 6, 1024)), ["s2", "t2", "r"], None, None, ["t2", "r"], "sum", "copy"),
        (rng.random((3, 4, 2048)), ["a3", "b3", "r3"], rng.random((4, 2048)), ["b3", "r3"], ["a3", "r3"], "max", "mul"),
    ]
    dev = [(E.to_device(A), la, None if B is None else E.to_device(B), lb, out, red, cmb)
           for A, la, B, lb, out, red, cmb in jobs]
    expect = [E.to_host(E.contract(A, la, B, lb, out, reduce=red, combine=cmb)) for A, la, B, lb, out, red, cmb in dev]
    G = E.to_device(rng.random((4, 5, 6)))
    gexp = E.to_host(E.gather(G, ["a", "b", "c"], {"b": 3}, ["c", "a"]))
    for graph in (False, True):
        prog = Program()
        prog.begin_batch()
        outs = [prog.contract(A, la, B, lb, out, reduce=red, combine=cmb) for A, la, B, lb, out, red, cmb in dev]
        gd, Aptr, gout = E.prepare_gather(G, ["a", "b", "c"], {"b": 3}, ["c", "a"])
        prog._keep.extend([gd, G, gout])
        ga = (ctypes.byref(gd), Aptr, None, N.ptr(gout), None)
        prog._batch.jobs.append(("gather", ga, ga))
        prog.end_batch()
        assert len(prog) == 1  # all seven jobs are small: one launch
        if graph:
            prog.capture()
        prog.run()
        for got, exp in zip(outs, expect):
            np.testing.assert_allclose(E.to_host(got), exp, rtol=1e-13, atol=0)
        np.testing.assert_array_equal(E.to_host(gout), gexp)
    # a batch of one is recorded as the plain launch
    prog = Program()
    prog.begin_batch()
    A, la, B, lb, out, red, cmb = dev[0]
    o = prog.contract(A, la, B, lb, out, reduce=red, combine=cmb)
    prog.end_batch()
    prog.run()
    np.testing.assert_allclose(E.to_host(o), expect[0], rtol=1e-13)


@pytest.mark.parametrize("red", [614400, 3 * 4099])
def test_long_contiguous_reduction_few_outputs(gpu, red):
    """A batched dot product (5 outputs, one long contiguous reduction — a packed greedy step):
    the planner cuts the run into chunks for split-K; sums match numpy to fp64 rounding."""
    from pgmpy_amd import engine as E

    rng = np.random.default_rng(9)
    A = rng.random((5, red))
    B = rng.random(red)
    got = E.to_host(E.contract(E.to_device(A), ["m", "k"], E.to_device(B), ["k"], ["m"], reduce="sum",
                               combine="mul"))
    np.testing.assert_allclose(got, A @ B, rtol=1e-12)


@pytest.mark.parametrize("rows", [64, 66, 1000, 1001])
def test_rows2_product_and_marginal_paths(gpu, rows):
    """Batched-BP shapes (rows innermost): even row counts take the 16-B two-rows-per-lane kernels
    (k_productn_rows2, k_contract_rows_tab2), odd counts and misaligned views the 8-B ones."""
    from pgmpy_amd import _native as NN

    E = _e()
    rng = np.random.default_rng(rows)
    psi = rng.random((4, 2, 3, 5))                      # no row axis (broadcast over rows)
    m1 = rng.random((4, 5, rows))
    m2 = rng.random((2, 3, rows))
    m2[0, 0, :7] = 0.0
    den = rng.random((2, 3, rows))
    den[0, 0, :7] = 0.0                                 # 0/0 -> 0
    den[1, 2, :3] = 0.0                                 # x/0 -> inf
    ops = [(E.to_device(psi), ["a", "b", "c", "d"]), (E.to_device(m1), ["a", "d", "r"]),
           (E.to_device(m2), ["b", "c", "r"]), (E.to_device(den), ["b", "c", "r"])]
    got = E.to_host(E.product_n(ops, ["a", "b", "c", "d", "r"],
                                kinds=[NN.PRODN_MUL, NN.PRODN_MUL, NN.PRODN_RATIO, NN.PRODN_DEN]))
    with np.errstate(divide="ignore", invalid="ignore"):
        q = m2 / den
    q[np.isnan(q)] = 0
    ref = np.einsum("abcd,adr,bcr->abcdr", psi, m1, q)
    np.testing.assert_allclose(got, ref, rtol=1e-14)
    # separator marginals of the product (short reductions) and a misaligned (offset) view
    B = E.to_device(ref)
    for keep, red in ((["b", "d", "r"], "sum"), (["a", "r"], "max"), (["c", "r"], "sum")):
        idx = {l: i for i, l in enumerate("abcdr")}
        full = ref.copy()
        full[~np.isfinite(full)] = 0.0
        Bf = E.to_device(full)
        axes = tuple(i for l, i in idx.items() if l not in keep)
        exp = full.sum(axis=axes) if red == "sum" else full.max(axis=axes)
        got = E.to_host(E.contract(Bf, list("abcdr"), None, None, keep, reduce=red, combine="copy"))
        np.testing.assert_allclose(got, exp, rtol=1e-13)
    import torch

    flat = torch.zeros(full.size + 1, dtype=torch.float64, device=B.device)
    view = flat[1:].view(full.shape)                    # 8-B aligned only: the 8-B kernels
    view.copy_(E.to_device(full))
    got = E.to_host(E.contract(view, list("abcdr"), None, None, ["b", "d", "r"], reduce="sum", combine="copy"))
    np.testing.assert_allclose(got, full.sum(axis=(0, 2)), rtol=1e-13)


@pytest.mark.parametrize("rows,red", [(64, "sum"), (200, "sum"), (200, "max"), (201, "sum"), (30, "sum")])
def test_product_n_marginal_fused(gpu, rows, red):
    """pgm_product_n_marginal: the clique product and its separator marginal in one pass (fused
    when rows are innermost with an even count >= 64; product_n + contract otherwise), including
    the in-place ratio update beta *= sigma / mu (0/0 -> 0) of the distribute sweep."""
    import torch

    from pgmpy_amd import _native as NN

    E = _e()
    rng = np.random.default_rng(rows)
    cl = list("abcdef")
    card = dict(zip(cl, (8, 2, 3, 8, 5, 9)))  # 576 kept states: enough blocks for the fused kernel
    sh = [card[v] for v in cl]
    psi = rng.random(sh)
    msg = rng.random([card["a"], card["c"], card["f"], rows])
    R = E.ROW
    fused = E.prepare_product_n_marginal([(E.to_device(psi), cl), (E.to_device(msg), ["a", "c", "f", R])],
                                         cl + [R], ["a", "d", "f", R])[-1]
    assert fused == (rows % 2 == 0 and rows >= 64)
    C, M = E.product_n_marginal([(E.to_device(psi), cl), (E.to_device(msg), ["a", "c", "f", R])], cl + [R],
                                ["a", "d", "f", R], reduce=red)
    full = psi[..., None] * msg[:, None, :, None, None, :, :]
    np.testing.assert_array_equal(E.to_host(C), full)
    exp = full.sum(axis=(1, 2, 4)) if red == "sum" else full.max(axis=(1, 2, 4))
    np.testing.assert_allclose(E.to_host(M), exp, rtol=1e-13)
    # in place: beta *= sigma / mu with zeros, marginal onto (a, d, f)
    beta = E.to_device(full)
    sig = rng.random([card["a"], card["d"], card["f"], rows])
    mu = rng.random([card["a"], card["d"], card["f"], rows])
    sig[0, 0, 0, :5] = 0.0
    mu[0, 0, 0, :5] = 0.0
    C2, M2 = E.product_n_marginal([(beta, cl + [R]), (E.to_device(sig), ["a", "d", "f", R]),
                                   (E.to_device(mu), ["a", "d", "f", R])], cl + [R], ["a", "d", "f", R], out=beta,
                                  kinds=[NN.PRODN_MUL, NN.PRODN_RATIO, NN.PRODN_DEN], reduce=red)
    assert C2.data_ptr() == beta.data_ptr()
    with np.errstate(divide="ignore", invalid="ignore"):
        q = sig / mu
    q[np.isnan(q)] = 0
    upd = full * q[:, None, None, :, None, :, :]
    np.testing.assert_allclose(E.to_host(beta), upd, rtol=1e-15)
    exp2 = upd.sum(axis=(1, 2, 4)) if red == "sum" else upd.max(axis=(1, 2, 4))
    np.testing.assert_allclose(E.to_host(M2), exp2, rtol=1e-13)
    torch.cuda.synchronize()


@pytest.mark.parametrize("rows,red,store", [(1000, "sum", True), (2048, "sum", True), (2100, "max", True),
                                            (2100, "sum", False), (4000, "sum", True)])
def test_product_n_marginal_bound_matches_generic(gpu, rows, red, store):
    """pgm_product_n_marginal_bind: the plan compiled into a specialised kernel gives the generic
    fused kernel's C bit for bit and M to 1e-14 (same product and reduction order; only FMA
    contraction may differ): row tails (rows/2 not a
    multiple of the block's row pairs), 1 and 2 row pairs per lane, max-product, marginal only, and
    the in-place ratio update beta *= sigma / mu (0/0 -> 0) with operands that lack the row axis."""
    import ctypes

    import torch

    from pgmpy_amd import _native as NN

    E = _e()
    L = NN.lib()
    rng = np.random.default_rng(rows)
    cl = list("abcdef")
    card = dict(zip(cl, (8, 2, 3, 8, 5, 9)))
    sh = [card[v] for v in cl]
    R = E.ROW
    psi = E.to_device(rng.random(sh))
    msg = E.to_device(rng.random([card["a"], card["c"], card["f"], rows]))
    sig = rng.random([card["a"], card["d"], card["f"], rows])
    mu = rng.random([card["a"], card["d"], card["f"], rows])
    sig[0, 0, 0, :5] = 0.0
    mu[0, 0, 0, :5] = 0.0
    sig, mu = E.to_device(sig), E.to_device(mu)
    red_c = E._REDUCE[red]

    def both(ops, marg, kinds=None, inplace=None):
        outs = []
        for bound_path in (False, True):
            base = inplace.clone() if inplace is not None else None
            o = [(base, ls) if t is inplace else (t, ls) for t, ls in ops]
            d, ptrs, C, ms, M, ok = E.prepare_product_n_marginal(o, cl + [R], marg, base, kinds, store)
            assert ok
            args = (ctypes.byref(d), ptrs, NN.ptr(C) if store else None, ms, red_c, NN.ptr(M))
            s = NN.stream_handle()
            if bound_path:
                b = ctypes.c_void_p()
                NN.check(L.pgm_product_n_marginal_bind(*args, ctypes.byref(b)), "bind")
                assert b.value, "shape above the specialisation threshold must bind"
                NN.check(L.pgm_pm_bound_run(b, s), "run")
                torch.cuda.synchronize()
                L.pgm_pm_bound_destroy(b)
            else:
                NN.check(L.pgm_product_n_marginal(*args, s), "generic")
            outs.append((E.to_host(C) if store else None, E.to_host(M)))
        (c0, m0), (c1, m1) = outs
        if store:
            np.testing.assert_array_equal(c1, c0)
        # same summation order; the generic kernel may fuse a product into the running sum (FMA)
        np.testing.assert_allclose(m1, m0, rtol=1e-14, atol=0)
        return c0, m0

    c0, m0 = both([(psi, cl), (msg, ["a", "c", "f", R])], ["a", "d", "f", R])
    if store:
        full = E.to_host(psi)[..., None] * E.to_host(msg)[:, None, :, None, None, :, :]
        np.testing.assert_array_equal(c0, full)
    beta = E.to_device(rng.random(sh + [rows]))
    both([(beta, cl + [R]), (sig, ["a", "d", "f", R]), (mu, ["a", "d", "f", R])], ["a", "d", "e", R],
         kinds=[NN.PRODN_MUL, NN.PRODN_RATIO, NN.PRODN_DEN], inplace=beta)
    both([(psi, cl), (sig, ["a", "d", "f", R]), (mu, ["a", "d", "f", R]), (msg, ["a", "c", "f", R])],
         ["a", "c", "e", "f", R], kinds=[NN.PRODN_MUL, NN.PRODN_RATIO, NN.PRODN_DEN, NN.PRODN_MUL])


@pytest.mark.parametrize("red", ["sum", "max"])
def test_marginal_only_psi_tile_matches_generic(gpu, red):
    """r05: a marginal-only pass whose kept dims include some that only psi carries walks the largest of
    them inside the block (its states share the loaded child messages; PMSpec.tdim) — the shape of C4's
    32,256-state clique sending its message to the root: psi over (g, h, i, j, k, F), two child messages
    over (h, k, F, rows), the message over (g, h, i, j, F, rows).  Equals the generic fused kernel (same
    product and summation order) to 1e-14, and the source shows the tile (two accumulator sets)."""
    import ctypes

    import torch

    from pgmpy_amd import _native as NN

    E = _e()
    L = NN.lib()
    rng = np.random.default_rng(5)
    cl = list("ghijkF")
    card = dict(zip(cl, (4, 2, 4, 4, 4, 63)))
    R, rows = E.ROW, 2000
    psi = E.to_device(rng.random([card[v] for v in cl]))
    m1 = E.to_device(rng.random([card["h"], card["k"], card["F"], rows]))
    m2 = E.to_device(rng.random([card["h"], card["k"], card["F"], rows]))
    ops = [(psi, cl), (m1, ["h", "k", "F", R]), (m2, ["h", "k", "F", R])]
    marg = ["g", "h", "i", "j", "F", R]
    outs = []
    for bound_path in (False, True):
        d, ptrs, C, ms, M, ok = E.prepare_product_n_marginal(ops, cl + [R], marg, None, None, False)
        assert ok
        args = (ctypes.byref(d), ptrs, None, ms, E._REDUCE[red], NN.ptr(M))
        s = NN.stream_handle()
        if bound_path:
            buf = ctypes.create_string_buffer(1 << 20)
            assert L.pgm_product_n_marginal_source(*args, buf, len(buf)) > 0
            assert b"a0t1" in buf.value, "the psi-only dims are walked inside the block"
            b = ctypes.c_void_p()
            NN.check(L.pgm_product_n_marginal_bind(*args, ctypes.byref(b)), "bind")
            assert b.value
            NN.check(L.pgm_pm_bound_run(b, s), "run")
            torch.cuda.synchronize()
            L.pgm_pm_bound_destroy(b)
        else:
            NN.check(L.pgm_product_n_marginal(*args, s), "generic")
        outs.append(E.to_host(M))
    np.testing.assert_allclose(outs[1], outs[0], rtol=1e-14, atol=0)
    h = {v: E.to_host(t) for v, t in (("psi", psi), ("m1", m1), ("m2", m2))}
    full = h["psi"][..., None] * h["m1"][None, :, None, None, :, :, :] * h["m2"][None, :, None, None, :, :, :]
    exp = full.sum(axis=4) if red == "sum" else full.max(axis=4)
    np.testing.assert_allclose(outs[1], exp, rtol=1e-12)


def test_bp_fused_marginals_many_rows(gpu):
    """Batched BP with >= 64 evidence rows takes the fused belief + separator-marginal kernels;
    calibrated beliefs must equal the unfused schedule's (single-row calibrations)."""
    import pandas as pd

    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.inference.EliminationOrder import junction_tree_from_model
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import codes_to_frame, forward_sample_codes

    m = get_example_model("pathfinder")
    bjt = BatchedJunctionTree(junction_tree_from_model(m))
    leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)
    codes, nodes = forward_sample_codes(m, 128, seed=3)
    df = codes_to_frame(m, codes, nodes, columns=leaves[:6])
    cal = bjt.calibrate_frame(df)
    assert any("product_n_marginal" in n for n in bjt.schedule(128, list(df.columns)).prog.notes)
    for r in (0, 77, 127):
        one = bjt.calibrate_frame(df.iloc[[r, r]].reset_index(drop=True))  # 2 rows: unfused kernels
        for c in bjt.cliques:
            np.testing.assert_allclose(cal.clique_belief(c, r), one.clique_belief(c, 0), rtol=1e-11, atol=1e-300)


def test_batch_product_n_jobs(gpu):
    """pgm_batch_add_product_n: a levelled Program runs independent n-ary products (MUL and the
    RATIO/DEN pair, broadcast and in-place operands) as ONE batched launch; results equal the
    single-launch kernel bit for bit (same multiplication order)."""
    from pgmpy_amd import _native as NN
    from pgmpy_amd.program import Program

    E = _e()
    rng = np.random.default_rng(11)
    a = E.to_device(rng.random((3, 4, 100)))
    b = E.to_device(rng.random((4, 100)))
    c = E.to_device(rng.random((3,)))
    x = E.to_device(rng.random((5, 64)))
    n_ = rng.random((5, 64))
    d_ = rng.random((5, 64))
    n_[0, :7] = 0.0
    d_[0, :7] = 0.0
    nn, dd = E.to_device(n_), E.to_device(d_)
    ref1 = E.to_host(E.product_n([(a, ["x", "y", "r"]), (b, ["y", "r"]), (c, ["x"])], ["y", "x", "r"]))
    x_before = E.to_host(x)
    ref2 = E.to_host(E.product_n([(x, ["a", "r"]), (nn, ["a", "r"]), (dd, ["a", "r"])], ["a", "r"],
                                 kinds=[NN.PRODN_MUL, NN.PRODN_RATIO, NN.PRODN_DEN]))
    prog = Program(levels=True)
    o1 = prog.product_n([(a, ["x", "y", "r"]), (b, ["y", "r"]), (c, ["x"])], ["y", "x", "r"])
    prog.product_n([(x, ["a", "r"]), (nn, ["a", "r"]), (dd, ["a", "r"])], ["a", "r"], out=x,
                   kinds=[NN.PRODN_MUL, NN.PRODN_RATIO, NN.PRODN_DEN])
    o3 = prog.product_n([(o1, ["y", "x", "r"]), (c, ["x"])], ["x", "y", "r"])  # depends on o1: next level
    # odd innermost extent: the 8-B flat form (the others run two elements per lane, 16-B)
    e_ = rng.random((3, 7))
    o4 = prog.product_n([(E.to_device(e_), ["x", "q"]), (c, ["x"])], ["x", "q"])
    assert prog.n_levels == 2
    assert len(prog) == 2 and prog.notes[0].startswith("level batch of 3")
    prog.run()
    np.testing.assert_array_equal(E.to_host(o4), e_ * E.to_host(c)[:, None])
    np.testing.assert_array_equal(E.to_host(o1), ref1)
    np.testing.assert_array_equal(E.to_host(x), ref2)
    np.testing.assert_array_equal(E.to_host(o3), np.transpose(ref1, (1, 0, 2)) * E.to_host(c)[:, None, None])
    assert not np.array_equal(x_before, ref2)


def test_single_workgroup_level_chain_matches_numpy(gpu, monkeypatch):
    """A plain Program's consecutive tiny levels (batches of at most PGM_WG_CHAIN_BLOCKS blocks) run as
    ONE single-workgroup launch (pgm_batch_set_mode ONE_WORKGROUP / k_batch_wg_c): two interleaved chains
    of dependent contractions, a wide level in the middle that keeps its own launch, a chain after it;
    every level equals numpy, on repeated runs and through a captured HIP graph."""
    import torch

    import pgmpy_amd.program as P
    from pgmpy_amd.program import Program

    monkeypatch.setattr(P, "WG_CHAIN_BLOCKS", 4)  # the default since r04; pinned here
    monkeypatch.setattr(P, "CHAIN_TUNE", False)  # keep the chain whatever the timing (tested below)
    E = _e()
    rng = np.random.default_rng(11)
    n_a, n_b = 6, 5  # tiny levels before / after the wide one
    xs = [rng.random((16, 8)) for _ in range(2)]
    Ws = [[rng.random((16, 16)) / 8 for _ in range(n_a + 1 + n_b)] for _ in range(2)]
    wide = rng.random((16, 4096)) / 16  # the wide level: [16, 8] x [16, 4096] -> 32 K outputs
    prog = Program()
    cur = [E.to_device(x) for x in xs]
    outs, want = [], []
    h = [x.copy() for x in xs]
    for lv in range(n_a + 1 + n_b):
        prog.begin_batch()
        if lv == n_a:
            nxt = [prog.contract(cur[c], ["a", "r"], E.to_device(wide), ["a", "w"], ["r", "w"], reduce="sum")
                   for c in range(2)]
            hn = [hh.T @ wide for hh in h]
        else:
            W = [E.to_device(Ws[c][lv]) for c in range(2)]
            if lv == n_a + 1:  # back to [16, 8]: fold the wide axis
                nxt = [prog.contract(cur[c], ["r", "w"], E.to_device(wide), ["a", "w"], ["a", "r"], reduce="sum")
                       for c in range(2)]
                hn = [wide @ hh.T for hh in h]
            else:
                nxt = [prog.contract(W[c], ["b", "a"], cur[c], ["a", "r"], ["b", "r"], reduce="sum") for c in range(2)]
                hn = [Ws[c][lv] @ h[c] for c in range(2)]
        prog.end_batch()
        cur, h = nxt, hn
        outs.append(cur)
        want.append(h)
    prog.run()
    notes = list(prog.notes)
    assert any("in one workgroup" in n for n in notes), notes
    assert len(prog) < n_a + 1 + n_b, notes

    def check():
        torch.cuda.synchronize()
        for lv in range(len(outs)):
            for c in range(2):
                np.testing.assert_allclose(E.to_host(outs[lv][c]), want[lv][c], rtol=1e-12)

    check()
    for o in outs:
        for t in o:
            t.zero_()
    prog.run()
    prog.run()
    check()
    prog.capture()
    for o in outs:
        for t in o:
            t.zero_()
    prog.run()
    check()


@pytest.mark.parametrize("operation", ["marginalize", "maximize"])
def test_bp_levelled_schedule_matches_sequential(gpu, operation):
    """The levelled batched-BP schedule (one launch per dependency level for the small cliques)
    equals the one-launch-per-step schedule on pathfinder, 1,000 rows; and it launches far less."""
    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree, BPSchedule
    from pgmpy_amd.inference.EliminationOrder import junction_tree_from_model
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("pathfinder")
    bjt = BatchedJunctionTree(junction_tree_from_model(m))
    leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)
    rows = 1000
    codes, nodes = forward_sample_codes(m, rows, seed=7)
    pos = {v: i for i, v in enumerate(nodes)}
    ev = leaves[:4]
    import torch

    d = torch.as_tensor(np.ascontiguousarray(codes[[pos[v] for v in ev]]), device="cuda")
    seq = BPSchedule(bjt, rows, ev, operation, marginals=True, levels=False)
    lev = BPSchedule(bjt, rows, ev, operation, marginals=True, levels=True)
    assert len(lev.prog) < len(seq.prog) // 2, (len(lev.prog), len(seq.prog))
    c1 = seq.run(d)
    c2 = lev.run(d)
    torch.cuda.synchronize()
    for c in bjt.cliques:
        for r in (0, 500, 999):
            np.testing.assert_allclose(c2.clique_belief(c, r), c1.clique_belief(c, r), rtol=1e-11, atol=1e-300)
    if operation == "marginalize":
        for v in bjt.variables[:20]:
            np.testing.assert_allclose(c2.marginal(v), c1.marginal(v), rtol=1e-11, atol=1e-300)


def test_bp_levelled_findings_batch_flags_bad_codes(gpu):
    """Findings indicators of a levelled sweep run as ONE batched launch (pgm_batch_add_indicator);
    an out-of-range evidence code still sets the error flag (-> IndexError, test_Factor.py:555-565)."""
    import torch

    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.inference.EliminationOrder import junction_tree_from_model
    from pgmpy_amd.utils import get_example_model

    m = get_example_model("alarm")
    bjt = BatchedJunctionTree(junction_tree_from_model(m))
    leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)[:5]
    rows = 128
    sch = bjt.schedule(rows, leaves)
    assert not any(n.startswith("indicator") for n in sch.prog.notes)  # all inside level batches
    codes = torch.zeros((len(leaves), rows), dtype=torch.uint8, device="cuda")
    sch.run(codes)
    torch.cuda.synchronize()
    assert int(sch.err.item()) == 0
    codes[2, 7] = 77  # not a state of that variable
    sch.run(codes)
    torch.cuda.synchronize()
    assert int(sch.err.item()) != 0


def test_specialised_kernel_disk_cache(gpu, tmp_path):
    """Specialised kernels are written to the code-object cache (PGM_KERNEL_CACHE) on first use and
    loaded from it by a later process: same kernels, no new files, identical beliefs."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PGM_KERNEL_CACHE=str(tmp_path / "kc"))
    runs = []
    for _ in range(2):
        r = subprocess.run([sys.executable, os.path.join(root, "tests", "workers", "pm_cache.py")], cwd=root,
                           env=env, timeout=240, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    a, b = runs
    assert a["bound"] > 0 and a["files"] > 0, a  # merged steps compile as one kernel per level
    assert b["bound"] == a["bound"] and b["files"] == a["files"], (a, b)
    assert b["checksum"] == a["checksum"]


@pytest.mark.parametrize("rows", [1000, 2100])
def test_product_n_bound_matches_generic(gpu, rows):
    """pgm_product_n_bind (the n-ary product as a specialised step, no marginal) and the same step
    merged with a marginal-only step (pgm_pm_merge) give the generic kernels' outputs exactly."""
    import ctypes

    import torch

    from pgmpy_amd import _native as NN

    E = _e()
    L = NN.lib()
    rng = np.random.default_rng(rows + 1)
    cl = list("abcdef")
    card = dict(zip(cl, (8, 2, 3, 8, 5, 9)))
    R = E.ROW
    psi = E.to_device(rng.random([card[v] for v in cl]))
    msg = E.to_device(rng.random([card["a"], card["c"], card["f"], rows]))
    sig = E.to_device(rng.random([card["a"], card["d"], card["f"], rows]))
    ops = [(psi, cl), (msg, ["a", "c", "f", R]), (sig, ["a", "d", "f", R])]
    d0, p0, C0 = E.prepare_product_n(ops, cl + [R])
    NN.check(L.pgm_product_n(ctypes.byref(d0), p0, NN.ptr(C0), NN.stream_handle()), "product_n")
    d1, p1, C1 = E.prepare_product_n(ops, cl + [R])
    b = ctypes.c_void_p()
    NN.check(L.pgm_product_n_bind(ctypes.byref(d1), p1, NN.ptr(C1), ctypes.byref(b)), "bind")
    assert b.value
    # a marginal-only step of another product, merged with the product into one launch
    d2, p2, C2, ms2, M2, ok = E.prepare_product_n_marginal(ops[:2], cl + [R], ["a", "d", "f", R], store=False)
    assert ok
    b2 = ctypes.c_void_p()
    NN.check(L.pgm_product_n_marginal_bind(ctypes.byref(d2), p2, None, ms2, E._REDUCE["sum"], NN.ptr(M2),
                                           ctypes.byref(b2)), "bind2")
    assert b2.value
    arr = (ctypes.c_void_p * 2)(b.value, b2.value)
    m = ctypes.c_void_p()
    NN.check(L.pgm_pm_merge(arr, 2, ctypes.byref(m)), "merge")
    assert m.value
    NN.check(L.pgm_pm_bound_run(m, NN.stream_handle()), "run merged")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(E.to_host(C1), E.to_host(C0))
    full = E.to_host(psi)[..., None] * E.to_host(msg)[:, None, :, None, None, :, :]
    np.testing.assert_allclose(E.to_host(M2), full.sum(axis=(1, 2, 4)), rtol=1e-13)
    for h in (b, b2, m):
        L.pgm_pm_bound_destroy(h)


@pytest.mark.parametrize("rows,red,ratio", [(1000, "sum", False), (2100, "max", False), (1000, "sum", True)])
def test_two_marginals_one_pass(gpu, rows, red, ratio):
    """pgm_product_n_marginals_bind: two marginals of one product (dims kept by both, by one only,
    by neither) in one specialised pass equal numpy's sums / maxima of the full product, including a
    sigma/mu ratio pair (0/0 -> 0) and a row tail."""
    import ctypes

    import torch

    from pgmpy_amd import _native as NN

    E = _e()
    L = NN.lib()
    rng = np.random.default_rng(rows + 7)
    cl = list("abcdef")
    card = dict(zip(cl, (4, 2, 3, 2, 5, 33)))  # 165 states kept by both marginals: enough blocks
    R = E.ROW
    psi = rng.random([card[v] for v in cl])
    A = rng.random([card["a"], card["b"], card["f"], rows])
    B = rng.random([card["c"], card["d"], card["f"], rows])
    ops = [(E.to_device(psi), cl), (E.to_device(A), ["a", "b", "f", R]), (E.to_device(B), ["c", "d", "f", R])]
    full = psi[..., None] * A[:, :, None, None, None, :, :] * B[None, None, :, :, None, :, :]
    kinds = None
    if ratio:
        mu = rng.random([card["a"], card["b"], card["f"], rows])
        A[0, 0, 0, :3] = 0.0
        mu[0, 0, 0, :3] = 0.0
        ops = [ops[0], (E.to_device(A), ["a", "b", "f", R]), (E.to_device(mu), ["a", "b", "f", R]), ops[2]]
        kinds = [NN.PRODN_MUL, NN.PRODN_RATIO, NN.PRODN_DEN, NN.PRODN_MUL]
        with np.errstate(divide="ignore", invalid="ignore"):
            q = A / mu
        q[np.isnan(q)] = 0.0
        full = psi[..., None] * q[:, :, None, None, None, :, :] * B[None, None, :, :, None, :, :]
    m1, m2 = ["a", "b", "e", "f", R], ["c", "d", "e", "f", R]  # e, f: by both; a,b / c,d: by one each
    d, ptrs, C = E.prepare_product_n(ops, cl + [R], None, kinds)
    Ms, st = [], []
    for mg in (m1, m2):
        M = E.empty([int(C.shape[(cl + [R]).index(l)]) for l in mg])
        Ms.append(M)
        st.append((ctypes.c_int64 * 7)(*[int(M.stride(mg.index(l))) if l in mg else 0 for l in cl + [R]]))
    b = ctypes.c_void_p()
    NN.check(L.pgm_product_n_marginals_bind(ctypes.byref(d), ptrs, st[0], NN.ptr(Ms[0]), st[1], NN.ptr(Ms[1]),
                                            E._REDUCE[red], ctypes.byref(b)), "bind")
    assert b.value
    NN.check(L.pgm_pm_bound_run(b, NN.stream_handle()), "run")
    torch.cuda.synchronize()
    L.pgm_pm_bound_destroy(b)
    f = np.sum if red == "sum" else np.max
    np.testing.assert_allclose(E.to_host(Ms[0]), f(full, axis=(2, 3)), rtol=1e-13)
    np.testing.assert_allclose(E.to_host(Ms[1]), f(full, axis=(0, 1)), rtol=1e-13)




@pytest.mark.parametrize("spec", [True, False])
def test_specialised_contraction_batch_matches_numpy(gpu, monkeypatch, spec):
    """A plain Program's level batch of contractions through the plan-specialised kernel
    (pgm_batch_specialise, r05) and through the generic k_batch_c: one-lane-per-output jobs, lanes
    per output on a long reduction, output pairs with 16-B accesses, every combine (mul / add / div
    with 0/0 -> 0 / div_raw / copy) and reduce (sum / max / none) — each equals numpy, rtol 1e-12."""
    import pgmpy_amd.program as P
    from pgmpy_amd.program import Program

    monkeypatch.setattr(P, "BATCH_SPECIALISE", spec)
    E = _e()
    rng = np.random.default_rng(21)
    A1, B1 = rng.random((7, 5, 6)), rng.random((6, 9))
    A2, B2 = rng.random((3, 2000)), rng.random((2000,))
    A3, B3 = rng.random((4, 5, 8)), rng.random((4, 8))
    A4, B4 = rng.random((6, 64)), rng.random((6,))
    A5, B5 = rng.random((5, 6, 4)), rng.random((6, 4))
    A5[0, :3, :] = 0.0
    B5[:2, :] = 0.0
    A6 = rng.random((3, 4, 5, 2))
    A7, B7 = rng.random((8, 16)), rng.random((16,)) + 0.5
    prog = Program()
    prog.begin_batch()
    o1 = prog.contract(E.to_device(A1), ["a", "b", "r"], E.to_device(B1), ["r", "c"], ["a", "b", "c"], reduce="sum")
    o2 = prog.contract(E.to_device(A2), ["a", "r"], E.to_device(B2), ["r"], ["a"], reduce="sum")
    o3 = prog.contract(E.to_device(A3), ["a", "r", "x"], E.to_device(B3), ["a", "x"], ["a", "x"], reduce="max",
                       combine="add")
    o4 = prog.contract(E.to_device(A4), ["a", "x"], E.to_device(B4), ["a"], ["a", "x"], combine="mul")
    o5 = prog.contract(E.to_device(A5), ["q", "a", "x"], E.to_device(B5), ["a", "x"], ["q", "a", "x"], combine="div")
    o6 = prog.contract(E.to_device(A6), ["a", "b", "c", "d"], None, None, ["d", "b"], reduce="sum", combine="copy")
    o7 = prog.contract(E.to_device(A7), ["a", "x"], E.to_device(B7), ["x"], ["x", "a"], combine="div_raw")
    prog.end_batch()
    prog.run()
    import torch

    torch.cuda.synchronize()
    assert any(("specialised" in n) == spec for n in prog.notes), prog.notes
    with np.errstate(invalid="ignore", divide="ignore"):
        r5 = A5 / B5[None]
    r5[np.isnan(r5)] = 0.0
    checks = [(o1, np.einsum("abr,rc->abc", A1, B1)), (o2, A2 @ B2), (o3, (A3 + B3[:, None, :]).max(axis=1)),
              (o4, A4 * B4[:, None]), (o5, r5), (o6, A6.sum(axis=(0, 2)).T), (o7, (A7 / B7[None]).T)]
    for got, want in checks:
        np.testing.assert_allclose(E.to_host(got), want, rtol=1e-12, atol=0)



def test_chain_tuning_keeps_results(gpu, monkeypatch):
    """_tune_chains (r05): the same two-chain program with CHAIN_TUNE on times the single-workgroup chain
    against one launch per level before its first run, records both times and keeps the faster form;
    whichever it kept, every level equals numpy on repeated runs and through a captured graph."""
    import torch

    import pgmpy_amd.program as P
    from pgmpy_amd.program import Program

    monkeypatch.setattr(P, "WG_CHAIN_BLOCKS", 4)
    monkeypatch.setattr(P, "CHAIN_TUNE", True)
    E = _e()
    rng = np.random.default_rng(12)
    n = 7
    x = rng.random((16, 8))
    Ws = [rng.random((16, 16)) / 8 for _ in range(n)]
    prog = Program()
    cur, h, outs, want = E.to_device(x), x.copy(), [], []
    for lv in range(n):
        prog.begin_batch()
        cur = prog.contract(E.to_device(Ws[lv]), ["b", "a"], cur, ["a", "r"], ["b", "r"], reduce="sum")
        prog.end_batch()
        h = Ws[lv] @ h
        outs.append(cur)
        want.append(h)
    prog.run()
    t = prog.chain_tuning
    assert t["chained_us"] > 0 and t["per_level_us"] > 0, t
    chained = any("in one workgroup" in nt for nt in prog.notes)
    assert chained == (t["chained_us"] <= t["per_level_us"]), (t, list(prog.notes))

    def check():
        torch.cuda.synchronize()
        for lv in range(n):
            np.testing.assert_allclose(E.to_host(outs[lv]), want[lv], rtol=1e-12)

    check()
    for o in outs:
        o.zero_()
    prog.run()
    check()
    prog.capture()
    for o in outs:
        o.zero_()
    prog.run()
    check()


def test_program_direct_chain_and_eligibility(gpu):
    """r05: Program.bind_direct / run_direct — a plain program whose steps are all plan-specialised launches
    (here 6 dependent levels, the first a level of 130 jobs split into parts over the kernel-argument budget)
    runs as one AQL chain on a user-mode queue with the graph replay's results bit for bit; a program with a
    step that is not a specialised launch (a raw host-ordered step) does not qualify and says why."""
    import torch

    from pgmpy_amd.inference.plan import DirectQueue
    from pgmpy_amd.program import Program

    E = _e()
    rng = np.random.default_rng(21)
    dq = DirectQueue()
    prog = Program()
    NJ = 3000  # independent jobs x 3 pointers > 8,192 (the pointer table's limit): specialised in parts
    xs = [E.to_device(rng.random((8, 4))) for _ in range(NJ)]
    W = [E.to_device(rng.random((8, 8)) / 4) for _ in range(200)]
    prog.begin_batch()
    cur = [prog.contract(W[i % 200], ["b", "a"], xs[i], ["a", "r"], ["b", "r"], reduce="sum") for i in range(NJ)]
    prog.end_batch()
    for lv in range(5):
        prog.begin_batch()
        cur = [prog.contract(W[(i + lv) % 200], ["b", "a"], cur[i], ["a", "r"], ["b", "r"], reduce="sum")
               for i in range(0, len(cur), 2)]
        prog.end_batch()
    out = cur
    assert prog.bind_direct(dq), prog.direct_note
    assert any("parts" in n for n in prog.notes), list(prog.notes)
    prog.run_direct()
    got = [E.to_host(t).copy() for t in out]
    for t in out:
        t.zero_()
    torch.cuda.synchronize()
    prog.run()
    torch.cuda.synchronize()
    for a, t in zip(got, out):
        np.testing.assert_array_equal(a, E.to_host(t))
    bad = Program()
    bad.begin_batch()
    y = bad.contract(W[0], ["b", "a"], xs[0], ["a", "r"], ["b", "r"], reduce="sum")
    bad.end_batch()
    bad.raw_step(lambda s: None, "host-ordered no-op")
    assert not bad.bind_direct(dq)
    assert "not specialised" in bad.direct_note, bad.direct_note
    del y


def test_program_direct_chain_split_last_level(gpu):
    """a chain whose LAST step is a level split into parts over the kernel-argument budget. The
    parts after the first are independent packets, and only the chain's last packet carries the completion
    signal and the system-scope release.  pgm_dq_run_chain gives that packet the barrier bit whatever its
    flag, so run_direct returns only after every part has completed, and the host sees all of their
    outputs, bit for bit as the graph replay writes them."""
    import torch

    from pgmpy_amd.inference.plan import DirectQueue
    from pgmpy_amd.program import Program

    E = _e()
    rng = np.random.default_rng(23)
    dq = DirectQueue()
    prog = Program()
    NJ = 3000
    xs = [E.to_device(rng.random((8, 64))) for _ in range(NJ)]
    W = [E.to_device(rng.random((8, 8)) / 4) for _ in range(200)]
    prog.begin_batch()
    mid = [prog.contract(W[i % 200], ["b", "a"], xs[i], ["a", "r"], ["b", "r"], reduce="sum") for i in range(NJ)]
    prog.end_batch()
    prog.begin_batch()  # the last level: 3,000 jobs x 3 pointers > 8,192, specialised in parts
    out = [prog.contract(W[(i + 7) % 200], ["b", "a"], mid[i], ["a", "r"], ["b", "r"], reduce="sum") for i in range(NJ)]
    prog.end_batch()
    assert prog.bind_direct(dq), prog.direct_note
    assert "parts" in prog.notes[-1], list(prog.notes)
    want = [W[(i + 7) % 200] for i in range(NJ)]
    for rep in range(3):
        for t in out:
            t.zero_()
        torch.cuda.synchronize()
        prog.run_direct()
        got = [E.to_host(t).copy() for t in out]  # read right after the chain returned
        for i, g in enumerate(got):
            ref = E.to_host(want[i]) @ (E.to_host(W[i % 200]) @ E.to_host(xs[i]))
            np.testing.assert_allclose(g, ref, rtol=1e-12, err_msg=f"rep {rep} job {i}")
    for t in out:
        t.zero_()
    torch.cuda.synchronize()
    prog.run()
    torch.cuda.synchronize()
    for a, t in zip(got, out):
        np.testing.assert_array_equal(a, E.to_host(t))


def test_specialised_batch_pointer_table(gpu):
    """r06: a level batch over 512 pointers (4 KB of kernel arguments) is ONE specialised kernel that reads its
    pointers from a table in device memory (instead of parts, one packet each); graph replay and the direct
    chain give numpy's values."""
    import torch

    from pgmpy_amd.inference.plan import DirectQueue
    from pgmpy_amd.program import Program

    E = _e()
    rng = np.random.default_rng(29)
    prog = Program()
    xs = [E.to_device(rng.random((6, 10))) for _ in range(400)]
    W = [E.to_device(rng.random((5, 6))) for _ in range(400)]
    prog.begin_batch()  # 400 jobs x 3 pointers = 1,200
    out = [prog.contract(W[i], ["b", "a"], xs[i], ["a", "r"], ["b", "r"], reduce="sum") for i in range(400)]
    prog.end_batch()
    prog.begin_batch()
    tot = [prog.contract(out[i], ["b", "r"], None, None, ["r"], reduce="sum", combine="copy") for i in range(0, 400, 7)]
    prog.end_batch()
    assert prog.bind_direct(DirectQueue()), prog.direct_note
    assert prog.notes[0] == "specialised batch of 400", list(prog.notes)
    for run in ("direct", "graph"):
        for t in out + tot:
            t.zero_()
        torch.cuda.synchronize()
        prog.run_direct() if run == "direct" else prog.run()
        torch.cuda.synchronize()
        for i in range(400):
            np.testing.assert_allclose(E.to_host(out[i]), E.to_host(W[i]) @ E.to_host(xs[i]), rtol=1e-12)
        for k, i in enumerate(range(0, 400, 7)):
            np.testing.assert_allclose(E.to_host(tot[k]), (E.to_host(W[i]) @ E.to_host(xs[i])).sum(0), rtol=1e-12)


@pytest.mark.parametrize("chain", [False, True])
def test_contract_n_jobs_match_numpy(gpu, chain):
    """r06: n-ary contraction jobs (pgm_batch_add_contract_n, specialised kernel only): one level of a
    plain Program with a 3-operand sum over two labels (nested literal loops), an 8-operand job, a long
    reduction to few outputs (G lanes per output), a max-product, a broadcast product with no reduction
    and a transposed output; chain=True records two dependent levels of them so they run as the
    single-workgroup chain.  Each equals numpy's einsum (products as a left fold, rtol 1e-12)."""
    import torch

    from pgmpy_amd.program import Program

    E = _e()
    rng = np.random.default_rng(31)
    X = [rng.random((3, 4)), rng.random((4, 5)), rng.random((5, 2))]
    Y = [rng.random((2,)) + 0.1 for _ in range(7)] + [rng.random((2, 3))]
    Z = [rng.random((2, 900)), rng.random((900, 4)), rng.random((4,))]
    W = [rng.random((3, 6)), rng.random((6, 4)), rng.random((3,))]
    V = [rng.random((5,)), rng.random((7,))]
    T = [rng.random((4, 3, 2)), rng.random((2, 3))]
    prog = Program()
    prog.begin_batch()
    o1 = prog.contract_n([(E.to_device(X[0]), ["a", "b"]), (E.to_device(X[1]), ["b", "c"]),
                          (E.to_device(X[2]), ["c", "d"])], ["a", "d"])
    o2 = prog.contract_n([(E.to_device(y), ["p"]) for y in Y[:7]] + [(E.to_device(Y[7]), ["p", "q"])], ["q"])
    o3 = prog.contract_n([(E.to_device(Z[0]), ["a", "r"]), (E.to_device(Z[1]), ["r", "s"]),
                          (E.to_device(Z[2]), ["s"])], ["a"])
    o4 = prog.contract_n([(E.to_device(W[0]), ["a", "b"]), (E.to_device(W[1]), ["b", "c"]),
                          (E.to_device(W[2]), ["a"])], ["c"], reduce="max")
    o5 = prog.contract_n([(E.to_device(V[0]), ["i"]), (E.to_device(V[1]), ["j"])], ["j", "i"])
    prog.end_batch()
    if chain:
        prog.begin_batch()
        o6 = prog.contract_n([(o1, ["a", "d"]), (E.to_device(T[0]), ["x", "a", "d"]), (E.to_device(T[1]), ["d", "a"])],
                             ["x"])
        prog.end_batch()
        prog.begin_batch()
        o7 = prog.contract_n([(o6, ["x"]), (o3, ["a"])], ["a"])
        prog.end_batch()
    prog.run()
    torch.cuda.synchronize()
    assert all("specialised" in n or "levels in one workgroup" in n for n in prog.notes), prog.notes
    r1 = np.einsum("ab,bc,cd->ad", *X)
    r2 = np.einsum("p,p,p,p,p,p,p,pq->q", *Y)
    r3 = np.einsum("ar,rs,s->a", *Z)
    r4 = (W[0][:, :, None] * W[1][None, :, :] * W[2][:, None, None]).max(axis=(0, 1))
    r5 = np.outer(V[1], V[0])
    got = [(o1, r1), (o2, r2), (o3, r3), (o4, r4), (o5, r5)]
    if chain:
        r6 = np.einsum("ad,xad,da->x", r1, *T)
        got += [(o6, r6), (o7, np.einsum("x,a->a", r6, r3))]
    for o, r in got:
        np.testing.assert_allclose(E.to_host(o), r, rtol=1e-12, atol=0)


def test_fused_query_programs_match_unfused(gpu, monkeypatch):
    """r06: compiled single queries with the path's pairwise steps fused into n-ary jobs
    (contraction.fuse_path) — fewer dependency levels — equal the unfused programs (PGM_FUSE=0 path) on
    the C2 munin rows and alarm's 50 C1 patterns, rtol 1e-10; the fused C2 program has fewer launches."""
    import pgmpy_amd.inference.contraction as C
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from tests.goldens import load_json

    c2 = load_json("munin_c2_rows.json")
    c1 = load_json("alarm_queries.json")

    def run(fuse):
        monkeypatch.setattr(C, "FUSE", fuse)
        C._PATHS.clear()
        ve2 = VariableElimination(get_example_model("munin"))
        ve1 = VariableElimination(get_example_model("alarm"))
        out = [np.asarray(ve2.query_unnormalized(c2["variables"], r["evidence"]).values) for r in c2["rows"][:4]]
        out += [np.asarray(ve1.query(p["variables"], p["evidence"], show_progress=False).values) for p in c1["patterns"]]
        runner, = ve2._compiled.values()
        prog = runner.plan.__dict__["_q1"]["joint"][0]
        return out, len(prog._direct) if prog._direct else len(prog)

    fused, n_fused = run(True)
    plain, n_plain = run(False)
    for a, b in zip(fused, plain):
        np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-300)
    assert n_fused < n_plain, (n_fused, n_plain)
