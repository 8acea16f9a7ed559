#!/usr/bin/env python3
"""Probe: HIP graph memcpy nodes with torch-pinned host buffers (captured pgm_memcpy_h2d /
pgm_memcpy_d2h_async around a kernel).  Replays the graph with new host inputs and reports whether each
replay copies the CURRENT host data in and the result out (diagnostic for QueryRunner; r03g)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd import engine as E
    from pgmpy_amd.program import Program

    L = N.lib()
    hin = torch.zeros(8, dtype=torch.float64, pin_memory=True)
    hout = torch.zeros(8, dtype=torch.float64, pin_memory=True)
    din = torch.zeros(8, dtype=torch.float64, device="cuda")
    two = E.to_device(np.full(8, 2.0))
    prog = Program()
    prog.raw_step(lambda s: N.check(L.pgm_memcpy_h2d(N.ptr(din), ctypes.c_void_p(hin.data_ptr()), 64, s)), "h2d")
    dout = prog.contract(din, ["a"], two, ["a"], ["a"], combine="mul")
    prog.raw_step(lambda s: N.check(L.pgm_memcpy_d2h_async(ctypes.c_void_p(hout.data_ptr()), N.ptr(dout), 64, s)),
                  "d2h")
    prog.capture()
    res = []
    for rep in range(4):
        hin.numpy()[:] = np.arange(8) + 10 * rep
        hout.numpy()[:] = -1
        prog.run()
        N.check(L.pgm_stream_sync(N.stream_handle()))
        got = hout.numpy().copy()
        res.append((rep, bool(np.array_equal(got, 2 * (np.arange(8) + 10 * rep))), got[:3].tolist(),
                    E.to_host(din)[:3].tolist()))
    for r in res:
        print("replay", r, flush=True)


if __name__ == "__main__":
    main()
