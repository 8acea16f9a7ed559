"""Byte-range footprints of recorded launches and the hazard check of a Program.

A levelled Program (program.py) orders its launches by the buffers each one *declares* it reads and
writes (storage keys).  A launch that touches bytes it did not declare would be placed in the same
dependency level as a launch it conflicts with — two jobs of one batch launch running concurrently on
the same bytes — and nothing downstream would notice except as a wrong number.  This module
recomputes what every launch touches from the launch's own descriptor (strides x cardinalities of
every operand, the workspace, the evidence-code columns), independently of the declared lists, and
Program.check_hazards() verifies

  1. coverage: every byte range a launch reads lies in a buffer it declares (read or write), every
     range it writes in a buffer it declares written, and every range lies inside a buffer the program
     holds (a freed temporary would show up here);
  2. order: any two launches whose ranges overlap with at least one write are in different
     dependency levels, the later-recorded one in the later level (levelled Program); the jobs of one
     batch launch are pairwise free of such overlaps (plain Program).

Footprints are conservative intervals [lo, hi) per operand (the span of a strided view); the error
flags the gather / indicator kernels raise with an atomic OR are "atomic" ranges, not hazards.
"""

READ, WRITE, ATOMIC = "r", "w", "a"


def span(ptr, cards, strides, elem):
    """[lo, hi) bytes of the strided view at `ptr` (element strides, `elem` bytes per element)."""
    if not ptr:
        return None
    if any(int(c) <= 0 for c in cards):
        return None
    lo = hi = 0
    for c, s in zip(cards, strides):
        ext = (int(c) - 1) * int(s)
        if ext < 0:
            lo += ext
        else:
            hi += ext
    return (int(ptr) + lo * elem, int(ptr) + (hi + 1) * elem)


def _add(out, rng, mode):
    if rng is not None:
        out.append((rng[0], rng[1], mode))


def _pv(p):
    """Pointer value of a ctypes c_void_p / int / None."""
    if p is None:
        return 0
    v = getattr(p, "value", p)
    return int(v or 0)


def contract_foot(d, pA, pB, pC, pws=None, ws_bytes=0):
    """pgm_contract: C[keep] = REDUCE_red COMBINE(A, B) (ContractDesc, include/pgmhip.h)."""
    nk, nr = int(d.n_keep), int(d.n_red)
    kc = [int(d.keep_card[i]) for i in range(nk)]
    rc = [int(d.red_card[i]) for i in range(nr)]
    out = []
    _add(out, span(_pv(pA), kc + rc, [d.keep_sa[i] for i in range(nk)] + [d.red_sa[i] for i in range(nr)], 8), READ)
    _add(out, span(_pv(pB), kc + rc, [d.keep_sb[i] for i in range(nk)] + [d.red_sb[i] for i in range(nr)], 8), READ)
    _add(out, span(_pv(pC), kc, [d.keep_sc[i] for i in range(nk)], 8), WRITE)
    if _pv(pws) and ws_bytes:
        out.append((_pv(pws), _pv(pws) + int(ws_bytes), WRITE))
    return out


def contract_n_foot(d, ptrs, pC):
    """pgm_batch_add_contract_n: every operand read over the kept and reduced index space, C written
    over the kept space (pgm_contractn_desc)."""
    nk, nr = int(d.n_keep), int(d.n_red)
    kc = [int(d.keep_card[i]) for i in range(nk)]
    rc = [int(d.red_card[i]) for i in range(nr)]
    out = []
    for t in range(int(d.n_ops)):
        _add(out, span(_pv(ptrs[t]), kc + rc, [d.keep_s[t][i] for i in range(nk)] + [d.red_s[t][i] for i in range(nr)],
                       8), READ)
    _add(out, span(_pv(pC), kc, [d.keep_sc[i] for i in range(nk)], 8), WRITE)
    return out


def product_n_foot(d, ptrs, pout, store=True, marg=()):
    """pgm_product_n (+ _marginal / _marginals): operands read over the keep space, C written when
    stored, every marginal M (strides over the keep labels, 0 = reduced) written."""
    nk = int(d.n_keep)
    kc = [int(d.keep_card[i]) for i in range(nk)]
    out = []
    for i in range(int(d.n_ops)):
        _add(out, span(_pv(ptrs[i]), kc, [d.keep_s[i][k] for k in range(nk)], 8), READ)
    if store:
        _add(out, span(_pv(pout), kc, [d.keep_sc[k] for k in range(nk)], 8), WRITE)
    for ms, pM in marg:
        _add(out, span(_pv(pM), kc, [int(ms[k]) for k in range(nk)], 8), WRITE)
    return out


def gather_foot(d, pA, pcodes, pout, perr=None):
    """pgm_gather: A read at the kept and evidence axes; the evidence columns' codes [col * ld + row0,
    + n_rows) read; out written; the error flag raised atomically."""
    nk, ne = int(d.n_keep), int(d.n_ev)
    out = []
    kc = [int(d.keep_card[i]) for i in range(nk)]
    ksa = [0 if i == int(d.batch_dim) else int(d.keep_sa[i]) for i in range(nk)]
    _add(out, span(_pv(pA), kc + [int(d.ev_card[j]) for j in range(ne)],
                   ksa + [int(d.ev_stride[j]) for j in range(ne)], 8), READ)
    n_rows = kc[int(d.batch_dim)] if int(d.batch_dim) >= 0 else 1
    pc = _pv(pcodes)
    if pc and ne:
        for j in range(ne):
            lo = pc + int(d.ev_col[j]) * int(d.ld) + int(d.row0)
            out.append((lo, lo + n_rows, READ))
    _add(out, span(_pv(pout), kc, [int(d.keep_sc[i]) for i in range(nk)], 8), WRITE)
    if _pv(perr):
        out.append((_pv(perr), _pv(perr) + 4, ATOMIC))
    return out


def indicator_foot(pcodes, n_rows, card, pout, s_card, s_row, perr=None):
    out = []
    if _pv(pcodes) and n_rows:
        out.append((_pv(pcodes), _pv(pcodes) + int(n_rows), READ))
    _add(out, span(_pv(pout), [card, n_rows], [s_card, s_row], 8), WRITE)
    if _pv(perr):
        out.append((_pv(perr), _pv(perr) + 4, ATOMIC))
    return out


def view_foot(t, mode):
    """The whole strided view of a torch tensor (dense GEMM operands: every element is touched)."""
    if t is None or t.numel() == 0:
        return []
    r = span(t.data_ptr(), list(t.shape), list(t.stride()), t.element_size())
    return [(r[0], r[1], mode)] if r else []


def argmax_foot(pX, n_rows, row_len, s_row, s_elem, pout32):
    out = []
    _add(out, span(_pv(pX), [n_rows, row_len], [s_row, s_elem], 8), READ)
    if _pv(pout32):
        out.append((_pv(pout32), _pv(pout32) + 4 * int(n_rows), WRITE))
    return out


# ---------------------------------------------------------------------------- the check
def _storages(tensors):
    """Sorted [(lo, hi, key)] of the distinct storages behind `tensors` (key = storage data_ptr, the
    hazard identity program._key uses)."""
    seen = {}
    for t in tensors:
        if t is None or not hasattr(t, "untyped_storage"):
            continue
        st = t.untyped_storage()
        p = st.data_ptr()
        if p:
            seen[p] = max(seen.get(p, 0), st.nbytes())
    return sorted((p, p + n, p) for p, n in seen.items())


def _owner(stores, lo, hi):
    """Key of the storage holding [lo, hi), or None."""
    import bisect

    i = bisect.bisect_right(stores, (lo, float("inf"), 0)) - 1
    if i >= 0 and stores[i][0] <= lo and hi <= stores[i][1]:
        return stores[i][2]
    return None


def check(units, tensors, ordered):
    """units: [(name, foot, declared_reads, declared_writes, order_key)] in record order; tensors:
    every buffer the program holds.  ordered(i, j) -> True when unit j (recorded after i) is
    guaranteed to start after unit i completes.  Returns a list of violation strings."""
    stores = _storages(tensors)
    bad = []
    by_store = {}
    for i, (name, foot, rd, wr, _) in enumerate(units):
        rd, wr = set(rd), set(wr)
        for lo, hi, mode in foot:
            key = _owner(stores, lo, hi)
            if key is None:
                bad.append(f"[{i}] {name}: {mode} bytes [{lo:#x}, {hi:#x}) lie in no buffer the program holds")
                continue
            if mode == ATOMIC:
                continue
            if mode == WRITE and key not in wr:
                bad.append(f"[{i}] {name}: writes buffer {key:#x} it does not declare written")
            elif mode == READ and key not in rd and key not in wr:
                bad.append(f"[{i}] {name}: reads buffer {key:#x} it does not declare")
            by_store.setdefault(key, []).append((lo, hi, mode == WRITE, i))
    for key, rs in by_store.items():
        if not any(w for _, _, w, _ in rs):
            continue
        rs.sort()
        # sweep: every pair of overlapping ranges with a write and different units
        active = []
        for lo, hi, w, i in rs:
            active = [a for a in active if a[1] > lo]
            for alo, ahi, aw, ai in active:
                if ai == i or not (w or aw):
                    continue
                a, b = min(ai, i), max(ai, i)
                if not ordered(a, b):
                    kinds = "write/write" if (w and aw) else "read/write"
                    bad.append(f"[{a}] {units[a][0]} and [{b}] {units[b][0]}: {kinds} overlap on buffer "
                               f"{key:#x} without an ordering")
            active.append((lo, hi, w, i))
    return bad
