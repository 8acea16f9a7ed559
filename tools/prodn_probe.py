#!/usr/bin/env python3
"""Time pgm_product_n / pgm_contract on the batched-BP shapes of pathfinder's largest clique
(32,256 states x R evidence rows) with operand subsets, to locate the gap to the write floor.

    python tools/prodn_probe.py [R]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from bench import HipTimer
    from pgmpy_amd import _native as N
    from pgmpy_amd import engine as E

    R = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    rng = np.random.default_rng(0)
    cl = ["F20", "F41", "F44", "F72", "F84", "F85", "Fault"]
    card = {"F20": 4, "F41": 2, "F44": 2, "F72": 2, "F84": 4, "F85": 4, "Fault": 63}
    psi = E.to_device(rng.random([card[v] for v in cl]))
    msg_l = ["F20", "F41", "F44", "F72", "Fault"]
    msg = E.to_device(rng.random([card[v] for v in msg_l] + [R]))
    ones = E.to_device(np.ones(R))
    full = E.to_device(rng.random([card[v] for v in cl] + [R]))
    out = torch.empty_like(full)
    sep = ["F20", "F72", "F84", "F85", "Fault"]
    sig = E.to_device(rng.random([card[v] for v in sep] + [R]))
    mu = E.to_device(rng.random([card[v] for v in sep] + [R]))
    Rl = E.ROW
    nbytes = out.numel() * 8

    L = N.lib()

    def pn(ops, kinds=None):  # descriptor prepared once, only the launch timed
        import ctypes

        d, ptrs, o = E.prepare_product_n(ops, cl + [Rl], out, kinds)
        return lambda: N.check(L.pgm_product_n(ctypes.byref(d), ptrs, N.ptr(o), N.stream_handle()))

    def ct(A, la, keep):
        import ctypes

        d, o, ws, wsb = E.prepare_contract(A, la, None, None, keep, "sum", "copy", None)
        return lambda: N.check(L.pgm_contract(ctypes.byref(d), N.ptr(A), None, N.ptr(o), N.ptr(ws), wsb,
                                              N.stream_handle()))

    def t(name, fn, bytes_):
        for _ in range(2):
            fn()
        tm = HipTimer()
        tm.start()
        for _ in range(10):
            fn()
        us = tm.stop_ms() * 100
        print(json.dumps({"case": name, "us": round(us, 1), "TBps": round(bytes_ / us / 1e6, 2)}), flush=True)

    t("psi (no row) x ones", pn([(psi, cl), (ones, [Rl])]), nbytes)
    sm = E.to_device(rng.random((4, 4)))
    t("msg (row, broadcast F84,F85) x small[F84,F85]", pn([(msg, msg_l + [Rl]), (sm, ["F84", "F85"])]), nbytes)
    t("psi x msg (collect)", pn([(psi, cl), (msg, msg_l + [Rl])]), nbytes)
    t("full copy", pn([(full, cl + [Rl])]), 2 * nbytes)
    t("full x sigma/mu (update, out of place)",
      pn([(full, cl + [Rl]), (sig, sep + [Rl]), (mu, sep + [Rl])], [N.PRODN_MUL, N.PRODN_RATIO, N.PRODN_DEN]),
      2 * nbytes)
    t("marginal to sep (copy/sum)", ct(full, cl + [Rl], sep + [Rl]), nbytes)

    def pm(ops, marg, kinds=None, o=None):  # fused product + marginal
        import ctypes

        d, ptrs, o2, ms, M, ok = E.prepare_product_n_marginal(ops, cl + [Rl], marg + [Rl], o, kinds)
        assert ok
        return lambda: N.check(L.pgm_product_n_marginal(ctypes.byref(d), ptrs, N.ptr(o2), ms, E._REDUCE["sum"], N.ptr(M),
                                                        N.stream_handle()))

    t("fused psi x msg + marg to msg scope (collect)", pm([(psi, cl), (msg, msg_l + [Rl]), (ones, [Rl])], msg_l),
      nbytes)
    t("fused update in place + marg to sep", pm([(full, cl + [Rl]), (sig, sep + [Rl]), (mu, sep + [Rl])], sep,
                                              [N.PRODN_MUL, N.PRODN_RATIO, N.PRODN_DEN], full), 2 * nbytes)


if __name__ == "__main__":
    main()
