"""Fixed launch sequences with preallocated buffers, replayed or captured as one HIP graph.

A Program records device launches (pgm_contract / pgm_product_n / pgm_indicator
/ pgm_gather) with their descriptors, operand pointers and workspaces resolved
at build time; run() replays them (one ctypes call each) and capture() records
them into a HIP graph (pgm_graph_capture_*) so a whole compiled schedule — a
batched BP calibration, a fixed-shape contraction plan — is one launch.
"""
import ctypes

from . import _native as N
from . import engine as E


class Program:
    def __init__(self):
        self._steps = []
        self._keep = []
        self._graph = None
        self._stream = None

    # ------------------------------------------------------------------ recording
    def contract(self, A, la, B, lb, out_labels, reduce=None, combine="mul", out=None):
        d, out, ws, wsb = E.prepare_contract(A, la, B, lb, out_labels, reduce, combine, out)
        args = (ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(out), N.ptr(ws), wsb)
        self._keep.extend([d, A, B, out, ws])
        L = N.lib()
        self._steps.append(lambda s, a=args: N.check(L.pgm_contract(*a, s), "contract"))
        return out

    def product_n(self, operands, out_labels, out=None, kinds=None):
        ops = list(operands)
        kinds = list(kinds) if kinds is not None else [N.PRODN_MUL] * len(ops)
        L = N.lib()
        while len(ops) > N.PRODN_MAX_OPS:  # fold the surplus (plain MUL operands) into the output first
            cut = N.PRODN_MAX_OPS if kinds[N.PRODN_MAX_OPS - 1] != N.PRODN_RATIO else N.PRODN_MAX_OPS - 1
            out = self.product_n(ops[:cut], out_labels, out, kinds[:cut])
            ops = [(out, list(out_labels))] + ops[cut:]
            kinds = [N.PRODN_MUL] + kinds[cut:]
        d, ptrs, out = E.prepare_product_n(ops, out_labels, out, kinds)
        self._keep.extend([d, ptrs, out] + [t for t, _ in ops])
        args = (ctypes.byref(d), ptrs, N.ptr(out))
        self._steps.append(lambda s, a=args: N.check(L.pgm_product_n(*a, s), "product_n"))
        return out

    def indicator(self, codes_col, card, n_rows, err=None):
        out = E.empty([card, n_rows])
        L = N.lib()
        args = (N.ptr(codes_col), int(n_rows), int(card), N.ptr(out), int(out.stride(0)), int(out.stride(1)),
                N.ptr(err))
        self._keep.extend([codes_col, out, err])
        self._steps.append(lambda s, a=args: N.check(L.pgm_indicator(*a, s), "indicator"))
        return out

    def gather(self, A, la, evidence, out_labels, codes, ld, row0, n_rows, err=None):
        d, Aptr, out = E.prepare_gather(A, la, evidence, out_labels, codes, ld, row0, n_rows)
        L = N.lib()
        args = (ctypes.byref(d), Aptr, N.ptr(codes), N.ptr(out), N.ptr(err))
        self._keep.extend([d, A, codes, out, err])
        self._steps.append(lambda s, a=args: N.check(L.pgm_gather(*a, s), "gather"))
        return out

    def pair_gemm(self, A, la, B, lb, keep, shape):
        """Recorded dense step (engine.prepare_gemm): C over `keep`, offset table kept alive."""
        d, table, C = E.prepare_gemm(A, la, B, lb, keep, shape)
        L = N.lib()
        args = (ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(C))
        self._keep.extend([d, table, A, B, C])
        self._steps.append(lambda s, a=args: N.check(L.pgm_gemm(*a, s), "gemm"))
        return C

    def argmax(self, X, n_rows, row_len, s_row, s_elem, out32):
        L = N.lib()
        args = (N.ptr(X), int(n_rows), int(row_len), int(s_row), int(s_elem), None, N.ptr(out32))
        self._keep.extend([X, out32])
        self._steps.append(lambda s, a=args: N.check(L.pgm_argmax(*a, s), "argmax"))

    # ------------------------------------------------------------------ execution
    def run(self, stream=None):
        s = N.stream_handle(stream)
        if self._graph is not None:
            N.check(N.lib().pgm_graph_launch(self._graph, s), "graph_launch")
            return
        for step in self._steps:
            step(s)

    def capture(self):
        """Record the steps into one HIP graph (captured on a private stream)."""
        import torch

        if self._graph is not None:
            return
        L = N.lib()
        self._stream = torch.cuda.Stream()
        torch.cuda.current_stream().synchronize()
        s = N.stream_handle(self._stream)
        g = ctypes.c_void_p()
        N.check(L.pgm_graph_capture_begin(s), "graph_capture_begin")
        try:
            for step in self._steps:
                step(s)
        finally:
            N.check(L.pgm_graph_capture_end(s, ctypes.byref(g)), "graph_capture_end")
        self._graph = g

    def __len__(self):
        return len(self._steps)

    def __del__(self):
        g = getattr(self, "_graph", None)
        if g is not None and g.value:
            try:
                N.load_library().pgm_graph_destroy(g)
            except Exception:
                pass
