"""Label-based device operations over fp64 torch tensors, dispatched to libpgmhip.

Every factor operation of the hot path is one ``contract`` call: operands are
device tensors whose axes carry variable labels; the kernel walks the output
labels (keep loop) and the labels that appear only in the inputs (reduce loop)
using each operand's element strides, so broadcasting (absent label -> stride 0),
transposition and batching over evidence rows (a ``ROW`` label) need no copies.

This module replaces the reference's numpy calls (pgmpy/utils/compat_fns.py:
einsum L63-67, max L53-60, argmax L70-74) with the C-ABI of include/pgmhip.h.
"""
import ctypes
import functools
import threading

import numpy as np

from . import _native as N

ROW = "__row__"  # label of the evidence-row (batch) axis

# SURVEY.md §8(b) threading: the reference calls map_query from joblib threads on one shared
# object (DiscreteBayesianNetwork.py:871) and ctypes releases the GIL.  A first query of a pattern
# captures a HIP graph, and HIP rejects work on the legacy stream from another thread while a
# stream is capturing.  So the Python side takes a readers-writer lock, as §8(b) allows: the public
# inference entry points hold it SHARED (replays of compiled plans run concurrently; each compiled
# runner serialises only its own buffers), every HIP graph capture holds it EXCLUSIVELY.


class DeviceLock:
    """Re-entrant readers-writer lock with writer preference.

    A thread may nest shared holds, nest exclusive holds, and take shared inside exclusive.  A thread
    that holds it shared and asks for it exclusively gives its shared hold up while it waits (and gets
    it back when it releases the exclusive hold): so a capture inside a public call needs no upgrade,
    and the rule that avoids deadlock is that no other lock is held while waiting for the exclusive
    one (capture sites take it before any per-plan lock, PatternPlan.prepare_steps).
    `peak_readers` records the most threads ever inside at once (a test's evidence of overlap)."""

    def __init__(self):
        self._mu = threading.Lock()
        self._cv = threading.Condition(self._mu)
        self._readers = 0
        self._writer = None
        self._wdepth = 0
        self._waiting_writers = 0
        self._tls = threading.local()
        self.peak_readers = 0

    def _t(self):
        t = self._tls
        if not hasattr(t, "n"):
            t.n, t.counted = 0, False
        return t

    def acquire_shared(self):
        # r06: the uncontended path takes the plain mutex only (a nested hold not even that: its count is
        # thread-local), and a release notifies only when a writer waits for the last reader — a compiled
        # single query (C1 / C2) takes this pair once per call
        t = self._tls
        n = getattr(t, "n", 0)
        if n > 0:
            t.n = n + 1
            return
        me = threading.get_ident()
        with self._mu:
            if self._writer == me:
                t.n = 1
                if not hasattr(t, "counted"):
                    t.counted = False
                return
            while self._writer is not None or self._waiting_writers:
                self._cv.wait()
            self._readers += 1
            if self._readers > self.peak_readers:
                self.peak_readers = self._readers
            t.n, t.counted = 1, True

    def release_shared(self):
        t = self._tls
        n = t.n - 1
        t.n = n
        if n == 0 and t.counted:
            with self._mu:
                t.counted = False
                self._readers -= 1
                if self._readers == 0 and self._waiting_writers:
                    self._cv.notify_all()

    def acquire_exclusive(self):
        me, t = threading.get_ident(), self._t()
        with self._cv:
            if self._writer == me:
                self._wdepth += 1
                return
            if t.counted:  # give the shared hold up while waiting (no upgrade deadlock)
                t.counted = False
                self._readers -= 1
                self._cv.notify_all()
            self._waiting_writers += 1
            while self._writer is not None or self._readers > 0:
                self._cv.wait()
            self._waiting_writers -= 1
            self._writer, self._wdepth = me, 1

    def release_exclusive(self):
        t = self._t()
        with self._cv:
            self._wdepth -= 1
            if self._wdepth == 0:
                self._writer = None
                if t.n > 0:  # back to the shared hold it had before
                    t.counted = True
                    self._readers += 1
                self._cv.notify_all()

    def shared(self):
        return _Held(self.acquire_shared, self.release_shared)

    def exclusive(self):
        return _Held(self.acquire_exclusive, self.release_exclusive)


class _Held:
    __slots__ = ("_a", "_r")

    def __init__(self, a, r):
        self._a, self._r = a, r

    def __enter__(self):
        self._a()
        return self

    def __exit__(self, *exc):
        self._r()
        return False


device_lock = DeviceLock()


def serialized(fn):
    """Run `fn` holding device_lock shared (public entry points; re-entrant)."""

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        with device_lock.shared():
            return fn(*args, **kwargs)

    return wrapper


def serialized_instance(fn):
    """`serialized` plus the object's own re-entrant lock, for entry points that change the object's
    state (BeliefPropagation.query swaps self.model for the pruned model and back, calibrate overwrites
    the clique beliefs and replays one cached schedule's buffers): two threads on one such object run
    one after the other, threads on different objects still overlap.  The object lock is taken BEFORE
    the shared device hold, so a thread waiting for it holds no share of device_lock and cannot block
    a capture's exclusive hold (DeviceLock's one rule)."""

    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        lk = self.__dict__.get("_instance_lock")
        if lk is None:
            lk = self.__dict__.setdefault("_instance_lock", threading.RLock())
        with lk:
            with device_lock.shared():
                return fn(self, *args, **kwargs)

    return wrapper


_tls_stream = threading.local()


def thread_stream():
    """This thread's own HIP stream (a torch.cuda.Stream per thread and device, non-blocking): compiled
    single queries replay and wait on it, so concurrent threads neither order their launches behind
    each other nor wait for each other's work (a spin on the shared default stream waits for every
    thread's launches).  Created after the default stream has drained, so buffers that work queued
    there initialised are complete before the first launch on it."""
    import torch

    d = torch.cuda.current_device()
    per = getattr(_tls_stream, "by_dev", None)
    if per is None:
        per = _tls_stream.by_dev = {}
    s = per.get(d)
    if s is None:
        torch.cuda.current_stream().synchronize()
        s = per[d] = torch.cuda.Stream(device=d)
    return s


def exclusive(fn):
    """Run `fn` holding device_lock exclusively (HIP graph captures)."""

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        with device_lock.exclusive():
            return fn(*args, **kwargs)

    return wrapper

_REDUCE = {None: N.RED_NONE, "sum": N.RED_SUM, "max": N.RED_MAX}
_COMBINE = {"mul": N.COMBINE_MUL, "add": N.COMBINE_ADD, "div": N.COMBINE_DIV, "copy": N.COMBINE_COPY,
            "div_raw": N.COMBINE_DIV_RAW}


def _torch():
    import torch

    return torch


def device():
    torch = _torch()
    N.lib()  # raises NativeUnavailable without a GPU / library
    return torch.device("cuda", torch.cuda.current_device())


def to_device(arr):
    """Host numpy (any dtype castable to fp64) -> contiguous fp64 device tensor.

    The H2D copy goes through the library (pgm_memcpy_h2d) on the current stream."""
    torch = _torch()
    L = N.lib()
    a = np.ascontiguousarray(arr, dtype=np.float64)
    t = torch.empty(a.shape, dtype=torch.float64, device=device())
    if a.size:
        N.check(L.pgm_memcpy_h2d(N.ptr(t), a.ctypes.data_as(ctypes.c_void_p), a.nbytes, N.stream_handle()),
                "memcpy_h2d")
    return t


def to_device_i64(arr):
    """Host int64 array -> device int64 tensor (descriptor tables)."""
    torch = _torch()
    a = np.ascontiguousarray(arr, dtype=np.int64)
    t = torch.empty(a.shape, dtype=torch.int64, device=device())
    if a.size:
        N.check(N.lib().pgm_memcpy_h2d(N.ptr(t), a.ctypes.data_as(ctypes.c_void_p), a.nbytes, N.stream_handle()),
                "memcpy_h2d")
    return t


def to_device_raw(arr):
    """Host numpy array of any fixed-size dtype -> device tensor of the same dtype and shape."""
    torch = _torch()
    a = np.ascontiguousarray(arr)
    dt = {np.dtype(np.uint8): torch.uint8, np.dtype(np.int8): torch.int8, np.dtype(np.int32): torch.int32,
          np.dtype(np.int64): torch.int64, np.dtype(np.float64): torch.float64}[a.dtype]
    t = torch.empty(a.shape, dtype=dt, device=device())
    if a.size:
        N.check(N.lib().pgm_memcpy_h2d(N.ptr(t), a.ctypes.data_as(ctypes.c_void_p), a.nbytes, N.stream_handle()),
                "memcpy_h2d")
    return t


def to_host(t):
    """Device tensor -> numpy (C-order copy of its logical contents)."""
    L = N.lib()
    if not t.is_contiguous():
        t = copy(t)
    out = np.empty(tuple(t.shape), dtype=np.float64)
    if out.size:
        N.check(L.pgm_memcpy_d2h(out.ctypes.data_as(ctypes.c_void_p), N.ptr(t), out.nbytes, N.stream_handle()),
                "memcpy_d2h")
    return out


def empty(shape):
    torch = _torch()
    return torch.empty(tuple(int(s) for s in shape), dtype=torch.float64, device=device())


def scalar(x):
    return to_device(np.array(x, dtype=np.float64))


def prepare_contract(A, la, B, lb, out_labels, reduce=None, combine="mul", out=None):
    """Build (descriptor, out, workspace, ws_bytes) for C[out_labels] = REDUCE COMBINE(A, B).

    A/B: device fp64 tensors (any strides), la/lb: one label per axis (B may be
    None for combine="copy").  Labels absent from an operand broadcast (stride 0);
    labels absent from out_labels are reduced."""
    L = N.lib()
    la = list(la)
    lb = list(lb) if B is not None else []
    out_labels = list(out_labels)
    if len(la) != A.dim() or (B is not None and len(lb) != B.dim()):
        raise ValueError("label count does not match tensor rank")
    card = {}
    for t, ls in ((A, la), (B, lb)):
        if t is None:
            continue
        for d, l in enumerate(ls):
            c = int(t.shape[d])
            if card.setdefault(l, c) != c:
                raise ValueError(f"cardinality mismatch for {l!r}: {card[l]} vs {c}")
    for l in out_labels:
        if l not in card:
            raise ValueError(f"output label {l!r} not in any operand")
    red = [l for l in dict.fromkeys(la + lb) if l not in out_labels]
    if red and reduce is None:
        raise ValueError(f"labels {red} would be reduced but reduce=None")
    if len(out_labels) > N.PGM_MAX_DIMS or len(red) > N.PGM_MAX_DIMS:
        raise ValueError(f"too many dimensions ({len(out_labels)} kept, {len(red)} reduced; limit {N.PGM_MAX_DIMS})")
    if out is None:
        out = empty([card[l] for l in out_labels])
    elif tuple(out.shape) != tuple(card[l] for l in out_labels):
        raise ValueError("out has the wrong shape")

    def st(t, ls, l):
        if t is None or l not in ls:
            return 0
        return int(t.stride(ls.index(l)))

    d = N.ContractDesc()
    d.combine = _COMBINE[combine]
    d.reduce = _REDUCE[reduce] if red else N.RED_NONE
    d.n_keep = len(out_labels)
    d.n_red = len(red)
    for i, l in enumerate(out_labels):
        d.keep_card[i] = card[l]
        d.keep_sa[i] = st(A, la, l)
        d.keep_sb[i] = st(B, lb, l)
        d.keep_sc[i] = int(out.stride(i))
    for i, l in enumerate(red):
        d.red_card[i] = card[l]
        d.red_sa[i] = st(A, la, l)
        d.red_sb[i] = st(B, lb, l)
    ws_bytes = ctypes.c_size_t(0)
    N.check(L.pgm_contract_workspace(ctypes.byref(d), ctypes.byref(ws_bytes)), "contract")
    ws = empty([ws_bytes.value // 8]) if ws_bytes.value else None
    return d, out, ws, ws_bytes.value


def contract(A, la, B, lb, out_labels, reduce=None, combine="mul", out=None):
    """C[out_labels] = REDUCE_{labels not in out} COMBINE(A[la], B[lb]) (one pgm_contract call).

    Returns the output tensor (C-order over out_labels unless `out` is given)."""
    L = N.lib()
    d, out, ws, wsb = prepare_contract(A, la, B, lb, out_labels, reduce, combine, out)
    N.check(L.pgm_contract(ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(out), N.ptr(ws), wsb, N.stream_handle()),
            "contract")
    # ws may be freed here: torch's caching allocator is stream-ordered, so its memory is only
    # handed to work queued after these kernels on the same stream.
    return out


GEMM_MIN_M = GEMM_MIN_N = 16
GEMM_MIN_K = 1  # outer-product-like steps (few shared states) still write C as coalesced tiles
GEMM_MIN_FLOPS = 1 << 22


def _group_offsets(t, ls, group, card):
    """(offsets, stride): element offset of every index of `group` (labels, C-order over the group)
    in tensor t[ls]; stride is the single element stride when the group collapses, else -1."""
    off = np.zeros(1, dtype=np.int64)
    for l in group:
        st = int(t.stride(ls.index(l))) if l in ls else 0
        off = (off[:, None] + np.arange(card[l], dtype=np.int64)[None, :] * st).reshape(-1)
    if len(off) == 1:
        return off, 0
    d = np.diff(off)
    return off, (int(d[0]) if d[0] >= 0 and np.all(d == d[0]) else -1)


def gemm_shape(la, lb, keep, card, force=False):
    """Classify the pairwise step sum_{(la|lb) - keep} A[la] B[lb] as a dense GEMM.

    Returns (batch, M, N, K) label lists — batch: in both operands and kept; M: A only; N: B only;
    K: in both, summed — or None when it is not GEMM-shaped (a label summed out of one operand
    alone, M/N below 16 states, K below 8, or under 4 MFLOP unless force)."""
    sa, sb, sk = set(la), set(lb), set(keep)
    if len(sa) != len(la) or len(sb) != len(lb) or not sk <= (sa | sb):
        return None
    if any(l not in sk and l not in sb for l in la) or any(l not in sk and l not in sa for l in lb):
        return None
    batch = [l for l in la if l in sb and l in sk]
    Ms = [l for l in la if l not in sb]
    Ns = [l for l in lb if l not in sa]
    Ks = [l for l in la if l in sb and l not in sk]

    def prod(g):
        p = 1
        for l in g:
            p *= int(card[l])
        return p

    nb, m, n, k = prod(batch), prod(Ms), prod(Ns), prod(Ks)
    small = 2 * nb * m * n * k < GEMM_MIN_FLOPS and not force
    if k < GEMM_MIN_K or m < GEMM_MIN_M or n < GEMM_MIN_N or small:
        return None
    return batch, Ms, Ns, Ks


def gemm_orient(la, lb, shape):
    """Plan-time choice for a dense step of C-order operands A[la], B[lb]: which operand is the
    kernel's A (its K group is read along the lanes' k) and the output label order (batch + M + N,
    so C's innermost variable lies along the lanes).  Returns (swap, out_labels, shape') with shape'
    expressed for the kernel's (A, B)."""
    batch, Ms, Ns, Ks = shape
    score = (la[-1] in Ks) + (lb[-1] in Ns)
    score_sw = (lb[-1] in Ks) + (la[-1] in Ms)
    if score_sw > score:
        kset = set(Ks)
        return True, batch + Ns + Ms, (batch, Ns, Ms, [l for l in lb if l in kset])
    return False, batch + Ms + Ns, shape


def prepare_gemm(A, la, B, lb, keep, shape):
    """(desc, offset table, C) for the dense step `shape` = (batch, M, N, K) of A[la] x B[lb]
    (gemm_shape), C allocated C-order over `keep`.  The offset table (pgm_gemm_desc) addresses
    every operand layout directly."""
    la, lb, keep = list(la), list(lb), list(keep)
    card = {l: int(A.shape[i]) for i, l in enumerate(la)}
    for i, l in enumerate(lb):
        if card.setdefault(l, int(B.shape[i])) != int(B.shape[i]):
            raise ValueError(f"cardinality mismatch for {l!r}")
    batch, Ms, Ns, Ks = list(shape[0]), list(shape[1]), list(shape[2]), list(shape[3])
    # tile loads run along each operand's innermost (unit-stride) variable when it is the last of
    # its group: A along m (lane_order bit 0) or k, B along k (bit 1) or n.  The k enumeration order
    # is shared by A and B, so when only B is k-innermost its innermost variable goes last.
    def unit_label(T, ls):  # the variable stored with stride 1 (None if none)
        u = [l for i, l in enumerate(ls) if T.stride(i) == 1 and T.shape[i] > 1]
        return u[0] if u else None

    def last(g, l):
        return [x for x in g if x != l] + [l]

    ia, ib = unit_label(A, la), unit_label(B, lb)
    if ia is not None and ia in Ks:
        Ks = last(Ks, ia)
    elif ib is not None and ib in Ks:
        Ks = last(Ks, ib)
    if ia is not None and ia in Ms and keep[-1] not in Ms:  # (C's innermost variable keeps its order)
        Ms = last(Ms, ia)
    lane_order = (1 if (ia is not None and Ms and Ms[-1] == ia) else 0) | \
        (2 if (ib is not None and Ks and Ks[-1] == ib) else 0)
    C = empty([card[l] for l in keep])
    parts = [_group_offsets(A, la, batch, card), _group_offsets(B, lb, batch, card), _group_offsets(C, keep, batch, card),
             _group_offsets(A, la, Ms, card), _group_offsets(C, keep, Ms, card),
             _group_offsets(A, la, Ks, card), _group_offsets(B, lb, Ks, card),
             _group_offsets(B, lb, Ns, card), _group_offsets(C, keep, Ns, card)]
    table = to_device_i64(np.concatenate([o for o, _ in parts]))
    d = N.GemmDesc()
    d.batch, d.m, d.n, d.k = len(parts[0][0]), len(parts[3][0]), len(parts[7][0]), len(parts[5][0])
    d.offsets = table.data_ptr()
    for i, (_, st) in enumerate(parts):
        d.stride[i] = st
    d.lane_order = lane_order
    return d, table, C


def pair_gemm(A, la, B, lb, keep, force=False, shape=None):
    """sum over (la | lb) - keep of A[la] * B[lb] into a new C-order tensor over `keep`, on FP64
    MFMA (pgm_gemm) when the step is a dense GEMM (gemm_shape); None otherwise (the caller uses
    the generic fused contraction).  force=True skips only the minimum-work threshold (tests)."""
    if shape is None:
        card = {l: int(A.shape[i]) for i, l in enumerate(la)}
        card.update({l: int(B.shape[i]) for i, l in enumerate(lb)})
        shape = gemm_shape(list(la), list(lb), keep, card, force)
        if shape is None:
            return None
    d, table, C = prepare_gemm(A, la, B, lb, keep, shape)
    N.check(N.lib().pgm_gemm(ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(C), N.stream_handle()), "gemm")
    return C


def prepare_product_n(operands, out_labels, out=None, kinds=None):
    """Descriptor for C[out_labels] = prod_i X_i (broadcast, no reduction), up to 8 operands.

    kinds: per operand N.PRODN_MUL (default) or a N.PRODN_RATIO / N.PRODN_DEN pair
    (X_i / X_{i+1} with NaN -> 0)."""
    N.lib()
    out_labels = list(out_labels)
    if not 1 <= len(operands) <= N.PRODN_MAX_OPS:
        raise ValueError(f"product_n takes 1..{N.PRODN_MAX_OPS} operands")
    card = {}
    for t, ls in operands:
        if len(ls) != t.dim():
            raise ValueError("label count does not match tensor rank")
        for d, l in enumerate(ls):
            c = int(t.shape[d])
            if card.setdefault(l, c) != c:
                raise ValueError(f"cardinality mismatch for {l!r}")
            if l not in out_labels:
                raise ValueError(f"label {l!r} would need a reduction")
    if out is None:
        out = empty([card[l] for l in out_labels])
    d = N.ProductNDesc()
    d.n_ops = len(operands)
    d.n_keep = len(out_labels)
    for i, k in enumerate(kinds or []):
        d.op_kind[i] = int(k)
    for i, l in enumerate(out_labels):
        d.keep_card[i] = card[l]
        d.keep_sc[i] = int(out.stride(i))
        for t_i, (t, ls) in enumerate(operands):
            d.keep_s[t_i][i] = int(t.stride(list(ls).index(l))) if l in ls else 0
    ptrs = (ctypes.c_void_p * len(operands))(*[t.data_ptr() for t, _ in operands])
    return d, ptrs, out


def prepare_contract_n(operands, out_labels, reduce="sum", out=None):
    """(descriptor, operand pointers, out) for C[out_labels] = REDUCE over the other labels of
    prod_i X_i (pgm_contractn_desc, r06): several pairwise steps of a contraction path as one batch job.
    operands: (device fp64 tensor, labels) pairs, up to PRODN_MAX_OPS."""
    N.lib()
    out_labels = list(out_labels)
    if not 1 <= len(operands) <= N.PRODN_MAX_OPS:
        raise ValueError(f"contract_n takes 1..{N.PRODN_MAX_OPS} operands")
    card = {}
    for t, ls in operands:
        if len(ls) != t.dim():
            raise ValueError("label count does not match tensor rank")
        for dd, l in enumerate(ls):
            c = int(t.shape[dd])
            if card.setdefault(l, c) != c:
                raise ValueError(f"cardinality mismatch for {l!r}")
    for l in out_labels:
        if l not in card:
            raise ValueError(f"output label {l!r} not in any operand")
    red = [l for l in card if l not in out_labels]
    if len(out_labels) > N.PGM_MAX_DIMS or len(red) > N.PGM_MAX_DIMS:
        raise ValueError("too many dimensions")
    if out is None:
        out = empty([card[l] for l in out_labels])
    d = N.ContractNDesc()
    d.n_ops = len(operands)
    d.reduce = _REDUCE[reduce]
    d.n_keep = len(out_labels)
    d.n_red = len(red)

    def st(t, ls, l):
        return int(t.stride(list(ls).index(l))) if l in ls else 0

    for i, l in enumerate(out_labels):
        d.keep_card[i] = card[l]
        d.keep_sc[i] = int(out.stride(i))
        for j, (t, ls) in enumerate(operands):
            d.keep_s[j][i] = st(t, ls, l)
    for i, l in enumerate(red):
        d.red_card[i] = card[l]
        for j, (t, ls) in enumerate(operands):
            d.red_s[j][i] = st(t, ls, l)
    ptrs = (ctypes.c_void_p * len(operands))(*[t.data_ptr() for t, _ in operands])
    return d, ptrs, out


def product_n(operands, out_labels, out=None, kinds=None):
    L = N.lib()
    d, ptrs, out = prepare_product_n(operands, out_labels, out, kinds)
    N.check(L.pgm_product_n(ctypes.byref(d), ptrs, N.ptr(out), N.stream_handle()), "product_n")
    return out


def prepare_product_n_marginal(operands, out_labels, marg_labels, out=None, kinds=None, store=True, M=None):
    """(descriptor, operand pointers, C, marginal strides, M, fused?) for C = product_n(...) and
    M[marg_labels] = reduce of C over the other labels (pgm_product_n_marginal); marg_labels must
    be a subset of out_labels.  fused is False when the fused kernel does not apply.  store=False:
    M alone (C's buffer only describes the index space)."""
    d, ptrs, out = prepare_product_n(operands, out_labels, out, kinds)
    out_labels, marg_labels = list(out_labels), list(marg_labels)
    if any(l not in out_labels for l in marg_labels):
        raise ValueError("marginal labels must be output labels")
    if M is None:
        M = empty([int(out.shape[out_labels.index(l)]) for l in marg_labels])
    ms = (ctypes.c_int64 * len(out_labels))(*[int(M.stride(marg_labels.index(l))) if l in marg_labels else 0
                                               for l in out_labels])
    ok = bool(N.lib().pgm_product_n_marginal_ok(ctypes.byref(d), ptrs, N.ptr(out) if store else None, ms, N.ptr(M)))
    return d, ptrs, out, ms, M, ok


def product_n_marginal(operands, out_labels, marg_labels, out=None, kinds=None, reduce="sum"):
    """C = prod of operands over out_labels and M = reduce(C) onto marg_labels, in one pass when
    the fused kernel applies (else product_n then contract).  Returns (C, M)."""
    d, ptrs, out, ms, M, ok = prepare_product_n_marginal(operands, out_labels, marg_labels, out, kinds)
    L = N.lib()
    if ok:
        N.check(L.pgm_product_n_marginal(ctypes.byref(d), ptrs, N.ptr(out), ms, _REDUCE[reduce], N.ptr(M),
                                         N.stream_handle()), "product_n_marginal")
        return out, M
    N.check(L.pgm_product_n(ctypes.byref(d), ptrs, N.ptr(out), N.stream_handle()), "product_n")
    return out, contract(out, list(out_labels), None, None, list(marg_labels), reduce=reduce, combine="copy", out=M)


def copy(A, la=None, out_labels=None):
    la = list(range(A.dim())) if la is None else la
    out_labels = la if out_labels is None else out_labels
    return contract(A, la, None, None, out_labels, combine="copy")


def total(A):
    """Sum of all entries -> 0-d device tensor."""
    return contract(A, list(range(A.dim())), None, None, [], reduce="sum", combine="copy")


def normalize_(A):
    """A /= A.sum() in place (0/0 -> NaN as DiscreteFactor.normalize, DiscreteFactor.py:530)."""
    s = total(A)
    labels = list(range(A.dim()))
    contract(A, labels, s, [], labels, combine="div_raw", out=A)
    return A


def normalize_rows_(A, la, row_label=ROW):
    """Per-row normalize of a batched tensor: every label except row_label is summed."""
    s = contract(A, la, None, None, [row_label], reduce="sum", combine="copy")
    contract(A, la, s, [row_label], la, combine="div_raw", out=A)
    return A


def argmax_rows(A, la, row_label=None):
    """First-flat-index argmax over all labels but row_label (C-order of la minus row)."""
    torch = _torch()
    L = N.lib()
    if row_label is None:
        X = A if A.is_contiguous() else copy(A)
        out = torch.empty(1, dtype=torch.int64, device=X.device)
        n = X.numel()
        N.check(L.pgm_argmax(N.ptr(X), 1, n, n, 1, N.ptr(out), None, N.stream_handle()), "argmax")
        return out
    other = [l for l in la if l != row_label]
    X = contract(A, la, None, None, [row_label] + other, combine="copy")
    n_rows = X.shape[0]
    row_len = int(np.prod(X.shape[1:])) if X.dim() > 1 else 1
    out = torch.empty(n_rows, dtype=torch.int64, device=X.device)
    N.check(L.pgm_argmax(N.ptr(X), n_rows, row_len, row_len, 1, N.ptr(out), None, N.stream_handle()), "argmax")
    return out


def prepare_gather(A, la, evidence, out_labels, codes=None, ld=0, row0=0, n_rows=None):
    """(desc, A pointer, out) for gather(); see there."""
    la = list(la)
    static = {l: s for l, s in evidence.items() if codes is None or not isinstance(s, tuple)}
    dynamic = {l: s[1] for l, s in evidence.items() if codes is not None and isinstance(s, tuple)}
    card = {l: int(A.shape[i]) for i, l in enumerate(la)}
    base = 0
    for l, s in static.items():
        if not (0 <= int(s) < card[l]):
            raise IndexError(f"index {s} is out of bounds for axis with size {card[l]}")
        base += int(s) * int(A.stride(la.index(l)))
    keep_shape = []
    for l in out_labels:
        if l == ROW:
            keep_shape.append(int(n_rows))
        else:
            keep_shape.append(card[l])
    out = empty(keep_shape)
    d = N.GatherDesc()
    d.n_keep = len(out_labels)
    d.n_ev = len(dynamic)
    d.batch_dim = out_labels.index(ROW) if ROW in out_labels else -1
    d.ld = int(ld)
    d.row0 = int(row0)
    for i, l in enumerate(out_labels):
        d.keep_card[i] = keep_shape[i]
        d.keep_sa[i] = 0 if l == ROW else int(A.stride(la.index(l)))
        d.keep_sc[i] = int(out.stride(i))
    for j, (l, col) in enumerate(dynamic.items()):
        d.ev_col[j] = int(col)
        d.ev_stride[j] = int(A.stride(la.index(l)))
        d.ev_card[j] = card[l]
    return d, ctypes.c_void_p(A.data_ptr() + 8 * base), out


def gather(A, la, evidence, out_labels, codes=None, ld=0, row0=0, n_rows=None, err=None):
    """Evidence reduce.

    evidence: {label: state} (static) or {label: column} with `codes` (uint8
    device tensor [n_cols, ld]) giving per-row states; per-row gathers need
    ROW in out_labels.  Labels of A that are in `evidence` are dropped."""
    L = N.lib()
    torch = _torch()
    d, Aptr, out = prepare_gather(A, la, evidence, out_labels, codes, ld, row0, n_rows)
    own_err = err is None and d.n_ev > 0
    if own_err:
        err = torch.zeros(1, dtype=torch.int32, device=A.device)
    N.check(L.pgm_gather(ctypes.byref(d), Aptr, N.ptr(codes), N.ptr(out), N.ptr(err), N.stream_handle()), "gather")
    if own_err and int(err.item()) != 0:
        raise IndexError("evidence state code out of range for its variable")
    return out


def indicator(codes_col, card, n_rows, err=None):
    """[card, n_rows] 0/1 evidence indicator from a uint8 code column (255 = unobserved)."""
    L = N.lib()
    out = empty([card, n_rows])
    N.check(L.pgm_indicator(N.ptr(codes_col), int(n_rows), int(card), N.ptr(out), int(out.stride(0)),
                            int(out.stride(1)), N.ptr(err), N.stream_handle()), "indicator")
    return out
