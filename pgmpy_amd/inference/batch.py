"""Batched-evidence front end: DataFrame <-> uint8 codes, pattern grouping, result frames.

Replaces the per-row Python loops of DiscreteBayesianNetwork.predict (joblib
threads over map_query per unique row, DiscreteBayesianNetwork.py:866-910) and
predict_probability (iterrows + query, L962-989).  Rows are encoded once into
column-major uint8 state codes (255 = NaN / unobserved),
grouped by evidence pattern, and each pattern runs as one compiled device plan
(pgmpy_amd.inference.plan.PatternPlan).
"""
import ctypes
import os
import threading

import numpy as np

from .. import _native as N
from .. import engine as E
from .plan import PatternPlan

MISSING = N.PGM_EV_MISSING


def _lookup_codes(values, st):
    """int64 state numbers of an object array against the state list, -1 where not found: one pass of
    pandas' C object hash table (1.7 ms per 100k cells) instead of isna + Categorical (6+ ms)."""
    try:
        from pandas._libs import hashtable as ht

        table = ht.PyObjectHashTable(max(len(st), 1))
        table.map_locations(np.asarray(st, dtype=object))
        return np.asarray(table.lookup(values), dtype=np.int64)
    except Exception:  # private API moved: the public path
        import pandas as pd

        return np.asarray(pd.Categorical(values, categories=st).codes, dtype=np.int64)


def encode_frame(model, data, columns=None):
    """[n_cols, n_rows] uint8 codes of `data` (state names -> state numbers, NaN -> 255).

    Evidence ingestion: categorical columns remap their category codes
    (O(n) integer work); other columns take one hash-table lookup per cell against the variable's
    state names, and only the cells it misses are examined again (NaN -> 255; the reference's
    fallback from an unknown state name to the str() match, DiscreteFactor.py:589-597)."""
    import pandas as pd

    columns = list(data.columns) if columns is None else list(columns)
    states = model.states
    n = len(data)
    codes = np.empty((len(columns), n), dtype=np.uint8)
    for j, col in enumerate(columns):
        st = list(states[col])
        if len(st) >= MISSING:
            raise ValueError(f"variable {col} has {len(st)} states; uint8 codes hold at most 254")
        v = data[col]
        if isinstance(v.dtype, pd.CategoricalDtype):
            cats = list(v.cat.categories)
            lut = _lookup_codes(np.asarray(cats, dtype=object), st) if cats else np.zeros(0, dtype=np.int64)
            cc = np.asarray(v.cat.codes, dtype=np.int64)
            c = np.where(cc >= 0, lut[np.maximum(cc, 0)] if len(lut) else -1, -1)
            vals = None
        else:
            vals = v.to_numpy(dtype=object)
            c = _lookup_codes(vals, st)
        miss = np.nonzero(c < 0)[0]
        if len(miss):
            if vals is None:
                vals = v.to_numpy(dtype=object)
            sub = vals[miss]
            na = pd.isna(sub)
            c[miss[na]] = MISSING
            rest = miss[~na]
            if len(rest):
                # retry through str(): numeric frames against string state names (and vice versa)
                sm = {str(x): i for i, x in enumerate(st)}
                for i in rest:
                    k = sm.get(str(vals[i]))
                    if k is None:
                        raise KeyError(f"state: {vals[i]} is an unknown for variable: {col}. It must be one of {st}")
                    c[i] = k
        codes[j] = c.astype(np.uint8)
    return codes


_COL_KEY_SEED = 0x5eed_cafe  # fixed: pattern keys are comparable across calls


class Evidence:
    """A DataFrame's evidence on the device: uint8 state codes [n_cols, n] (255 = NaN) and the rows
    grouped by evidence pattern, [(observed column mask, row indices)]."""

    def __init__(self, codes, groups, n):
        self.codes, self.groups, self.n = codes, groups, n

    def rows_codes(self, rows):
        """Device codes of a subset of rows (one evidence pattern), [n_cols, len(rows)]."""
        import torch

        if len(rows) == self.n:
            return self.codes
        idx = torch.as_tensor(np.asarray(rows, dtype=np.int64), device=self.codes.device)
        return self.codes.index_select(1, idx).contiguous()


def _column_raw(v, st, col, fallback=None):
    """(int8 raw indices, LUT) of one column: pandas Categorical codes or Arrow dictionary indices
    and a category -> state LUT, or, for any other dtype, the state numbers themselves (one host hash
    pass) and the identity LUT.
    None when the column does not fit int8 indices (the host encoder handles the frame).  `fallback`
    (a set) receives `col` when a cell reached its state through the str() fallback."""
    import pandas as pd

    cats = raw = None
    if isinstance(v.dtype, pd.CategoricalDtype):
        cats = np.asarray(v.cat.categories, dtype=object)
        raw = v.cat.codes.to_numpy()
    elif isinstance(v.dtype, pd.ArrowDtype):
        import pyarrow as pa

        if pa.types.is_dictionary(v.dtype.pyarrow_dtype):  # Arrow dictionary-encoded column
            da = v.array.__arrow_array__().unify_dictionaries().combine_chunks()
            if not pa.types.is_int8(da.indices.type):
                return None
            cats = np.asarray(da.dictionary.to_pylist(), dtype=object)
            raw = np.asarray(da.indices.fill_null(-1).to_numpy(zero_copy_only=False), dtype=np.int8)
    if raw is not None:
        if raw.dtype != np.int8 or len(cats) > 127:
            return None
        lut = _lookup_codes(cats, st) if len(cats) else np.zeros(0, dtype=np.int64)
        miss = np.nonzero(lut < 0)[0]
        if len(miss):  # the reference's str() fallback per category; 254 = not a state name
            sm = {str(x): i for i, x in enumerate(st)}
            for i in miss:
                lut[i] = sm.get(str(cats[i]), 254)
            if fallback is not None:
                fallback.add(col)
        return raw, lut.astype(np.uint8)
    if len(st) > 127:
        return None
    vals = v.to_numpy(dtype=object)
    c = _lookup_codes(vals, st)
    miss = np.nonzero(c < 0)[0]
    if len(miss):
        sub = vals[miss]
        na = pd.isna(sub)
        c[miss[na]] = -1
        rest = miss[~na]
        if len(rest):
            sm = {str(x): i for i, x in enumerate(st)}
            for i in rest:
                k = sm.get(str(vals[i]))
                if k is None:
                    raise KeyError(f"state: {vals[i]} is an unknown for variable: {col}. It must be one of {st}")
                c[i] = k
            if fallback is not None:
                fallback.add(col)
    return c.astype(np.int8), np.arange(len(st), dtype=np.uint8)


def ingest_frame(model, data, columns=None, row_hash=False):
    """Evidence of a DataFrame on the device.

    Host: per column, its int8 category indices (pandas Categorical codes, zero-copy of the frame's
    own codes) or one hash pass for object columns, into a pinned [n_cols, n] buffer, plus a small
    category -> state LUT.  Device (pgm_codes_remap): one pass maps every cell to its uint8 state
    code and keys each row by its missing-column pattern; the host groups rows by (key, count)
    from 12 B per row.  Falls back to the host encoder (encode_frame) for variables with > 127
    states or categoricals with > 127 categories."""
    import torch

    columns = list(data.columns) if columns is None else list(columns)
    states = model.states
    n = len(data)
    nc = len(columns)
    raws, luts = [], []
    fallback = set()
    for col in columns:
        st = list(states[col])
        if len(st) >= MISSING:
            raise ValueError(f"variable {col} has {len(st)} states; uint8 codes hold at most 254")
        r = _column_raw(data[col], st, col, fallback)
        if r is None:
            codes = encode_frame(model, data, columns)
            ev = Evidence(upload_codes(codes), group_patterns(codes), n)
            ev.fallback_cols = None  # unknown: the host encoder does not report it
            if row_hash:
                ev.row_hash = _host_row_hash(codes)
            return ev
        raws.append(r[0])
        luts.append(r[1])
    L = N.lib()
    dev = E.device()
    s = N.stream_handle()
    h_raw = torch.empty((nc, n), dtype=torch.int8, pin_memory=True)
    hr = h_raw.numpy()
    for j, r in enumerate(raws):
        hr[j] = r
    lut = np.full((nc, 128), 254, dtype=np.uint8)
    for j, t in enumerate(luts):
        lut[j, :len(t)] = t
    keys = np.random.default_rng(_COL_KEY_SEED).integers(1, 2 ** 63, size=max(nc, 1), dtype=np.int64)
    d_raw = torch.empty((nc, n), dtype=torch.int8, device=dev)
    d_codes = torch.empty((nc, n), dtype=torch.uint8, device=dev)
    d_lut = E.to_device_raw(lut)
    d_key = E.to_device_raw(keys)
    d_rk = torch.zeros(n, dtype=torch.int64, device=dev)
    d_nm = torch.zeros(n, dtype=torch.int32, device=dev)
    d_hash = torch.zeros((n, 2), dtype=torch.int64, device=dev) if row_hash else None
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    if n and nc:
        N.check(L.pgm_memcpy_h2d(N.ptr(d_raw), ctypes.c_void_p(h_raw.data_ptr()), h_raw.numel(), s), "memcpy_h2d")
        N.check(L.pgm_codes_remap(N.ptr(d_raw), n, nc, n, N.ptr(d_lut), 128, N.ptr(d_key), N.ptr(d_codes), n,
                                  N.ptr(d_rk), N.ptr(d_nm), N.ptr(d_hash), N.ptr(err), s), "codes_remap")
    nm = download(d_nm)
    if int(download(err)[0]):
        encode_frame(model, data, columns)  # raises the reference's KeyError for the offending cell
        raise KeyError("evidence holds a category that is not a state name")
    if not nm.any():
        groups = [(np.ones(nc, dtype=bool), np.arange(n))]
    else:
        rk = download(d_rk)
        pair = np.stack([rk, nm.astype(np.int64)], axis=1)
        _, first, inv = np.unique(pair, axis=0, return_index=True, return_inverse=True)
        inv = inv.reshape(-1)
        order = np.argsort(inv, kind="stable")
        bounds = np.searchsorted(inv[order], np.arange(len(first) + 1))
        groups = []
        for g in range(len(first)):
            rows = order[bounds[g]:bounds[g + 1]]
            groups.append((hr[:, rows[0]] >= 0, rows))
        groups.sort(key=lambda gr: gr[1][0])
    ev = Evidence(d_codes, groups, n)
    ev.fallback_cols = fallback
    if row_hash:
        ev.row_hash = download(d_hash)
    return ev


_LUT_CACHE = {}  # (id(CategoricalDtype), variable) -> (dtype, state names, LUT, categories all valid)
_LUT_CACHE_MAX = 16384
_LUT_LOCK = threading.Lock()


def _category_lut(col, st, dtype):
    """(256-entry category index -> state code LUT, every category a state) of a categorical column
    (uint8 view of the int8 codes: index 255 is NaN -> MISSING; 254 = a category that is not a state
    name).  The reference's str() fallback applies per category (DiscreteFactor.py:589-597).  Cached
    per dtype object (a strong reference is kept, so its id is not reused while cached): frames
    built from one CategoricalDtype per variable, or the same frame again, pay this once."""
    key = (id(dtype), col)
    hit = _LUT_CACHE.get(key)
    if hit is not None and hit[0] is dtype and hit[1] == st:
        return hit[2], hit[3]
    cats = np.asarray(dtype.categories, dtype=object)
    t = _lookup_codes(cats, st) if len(cats) else np.zeros(0, dtype=np.int64)
    miss = np.nonzero(t < 0)[0]
    if len(miss):
        sm = {str(x): i for i, x in enumerate(st)}
        for i in miss:
            t[i] = sm.get(str(cats[i]), 254)
    lut = np.full(256, 254, dtype=np.uint8)
    lut[:len(t)] = t
    lut[255] = MISSING
    ok = not (t == 254).any()
    with _LUT_LOCK:
        if len(_LUT_CACHE) >= _LUT_CACHE_MAX:
            _LUT_CACHE.clear()
        _LUT_CACHE[key] = (dtype, list(st), lut, ok)
    return lut, ok


def _host_threads():
    """Host threads for native ingestion scans: the CPUs this process may run on, at most 16 (the GPU
    box's CPU share per GPU)."""
    import os

    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:  # pragma: no cover
        return max(1, min(16, os.cpu_count() or 1))


def _frame_categoricals(data, columns):
    """The pandas Categorical of every column, in `columns` order (one block per categorical column:
    read through the block manager, not per-column Series), or None."""
    import pandas as pd

    try:
        mgr = data._mgr
        arrays, blknos, blklocs = mgr.arrays, mgr.blknos, mgr.blklocs
        if len(columns) == len(data.columns) and all(a is b for a, b in zip(columns, data.columns)):
            loc = np.arange(len(columns))  # the frame's own column order (predict's call)
        else:
            loc = data.columns.get_indexer(columns)
            if (loc < 0).any():
                return None
        if len(loc) and np.asarray(blklocs)[loc].any():  # every column its own one-column block
            return None
        cat = pd.Categorical
        out = [arrays[b] for b in np.asarray(blknos)[loc].tolist()]
        if not all(type(a) is cat or isinstance(a, cat) for a in out):
            return None
        return out
    except Exception:  # pandas internals moved: the public accessor
        out = []
        for c in columns:
            a = data[c].array
            if not isinstance(a, pd.Categorical):
                return None
            out.append(a)
        return out


class ColumnarEvidence:
    """Evidence of a frame whose every column is categorical (pandas Categorical with <= 127
    categories): the int8 category codes stay in the frame (zero copy).  Rows are grouped by their
    missing-column pattern from the NaN-holding columns only (found by one native scan,
    pgm_host_any_negative_i8), and a pattern's plan gets just the columns it reads
    (PatternPlan.compact()), mapped through per-column LUTs and uploaded — a munin template frame
    (1,038 columns) moves 7 of them.  Replaces the per-row state-name lookups of predict /
    predict_probability (DiscreteBayesianNetwork.py:871-878, 974-979)."""

    def __init__(self, raws, luts, groups, n, addrs=None):
        self.raws, self.luts, self.groups, self.n = raws, luts, groups, n
        self._addrs = addrs  # column addresses while the NaN scan is pending (groups None)
        self._scan = None

    def start_scan(self):
        """Run the pending NaN scan on a worker thread (the native scan releases the GIL), so the caller
        can work on the device meanwhile; finish_scan() joins it and builds the groups."""
        if self.groups is not None or self._scan is not None:
            return
        has_nan = np.zeros(len(self.raws), dtype=np.uint8)
        box = {}

        def work():
            try:
                _scan_negative(self._addrs, self.n, has_nan)
            except BaseException as e:  # re-raised by finish_scan
                box["error"] = e

        t = threading.Thread(target=work, daemon=True)
        self._scan = (t, has_nan, box)
        t.start()

    def finish_scan(self):
        if self.groups is not None:
            return
        if self._scan is None:
            has_nan = np.zeros(len(self.raws), dtype=np.uint8)
            _scan_negative(self._addrs, self.n, has_nan)
        else:
            t, has_nan, box = self._scan
            t.join()
            self._scan = None
            if "error" in box:
                raise box["error"]
        self.groups = _nan_groups(self.raws, has_nan, self.n)
        self._addrs = None

    def host_codes_for(self, cols, rows):
        """uint8 state codes [len(cols), len(rows)] of the given frame columns and rows (host)."""
        full = len(rows) == self.n
        out = np.empty((len(cols), len(rows)), dtype=np.uint8)
        for i, j in enumerate(cols):
            r = self.raws[j].view(np.uint8)
            np.take(self.luts[j], r if full else r[rows], out=out[i])
        return out

    def codes_for(self, cols, rows):
        """The same codes on the device."""
        return upload_codes(self.host_codes_for(cols, rows))


def ingest_columnar(model, data, columns, defer_scan=False):
    """ColumnarEvidence of `data`, or None when a column is not a (small) pandas Categorical.
    Raises the reference's KeyError when a cell holds a category that is not a state name.
    defer_scan: leave the NaN scan (and so the groups) pending for ColumnarEvidence.start_scan /
    finish_scan."""
    if data.columns.has_duplicates:
        return None
    cats = _frame_categoricals(data, columns)
    if cats is None:
        return None
    n = len(data)
    fast = _schema_fast(model, columns, cats, n)
    if fast is not None:
        raws, luts, addrs = fast
        if defer_scan:
            return ColumnarEvidence(raws, luts, None, n, addrs)
        has_nan = np.zeros(len(columns), dtype=np.uint8)
        _scan_negative(addrs, n, has_nan)
        return ColumnarEvidence(raws, luts, _nan_groups(raws, has_nan, n), n)
    raws, luts, addrs = [], [], []
    all_ok = True
    i8 = np.dtype(np.int8)
    cpd_of = getattr(model, "_cpd_index", None) or {}
    addressof, char_at = ctypes.addressof, ctypes.c_char.from_buffer
    for col, arr in zip(columns, cats):
        try:
            raw = arr._codes  # the codes ndarray itself (the public .codes makes a read-only view per call)
        except AttributeError:  # pragma: no cover - pandas internals moved: the public accessor
            try:
                raw = arr.codes
            except (AttributeError, TypeError):
                return None  # the general encoder takes the frame
        if raw.dtype is not i8 or not raw.flags.c_contiguous:
            return None
        try:  # the buffer protocol's address: ~5x cheaper than building __array_interface__ per column
            addrs.append(addressof(char_at(raw)) if n else 0)
        except (TypeError, ValueError):  # a read-only or empty buffer
            addrs.append(raw.__array_interface__["data"][0])
        cpd = cpd_of.get(col)
        if cpd is None:
            cpd = model.get_cpds(col)  # raises the reference's error for a column that is not a node
        st = cpd.state_names[col]
        if len(st) >= MISSING:
            raise ValueError(f"variable {col} has {len(st)} states; uint8 codes hold at most 254")
        lut, ok = _category_lut(col, st, arr.dtype)
        if not ok:
            all_ok = False
            bad = np.nonzero(lut[:len(arr.dtype.categories)] == 254)[0]
            if np.isin(raw, bad.astype(np.int8)).any():
                encode_frame(model, data, [col])  # raises the reference's KeyError for the cell
                raise KeyError(f"evidence holds a category of {col} that is not a state name")
        raws.append(raw)
        luts.append(lut)
    if all_ok:
        _schema_store(model, columns, cats, luts)
    if defer_scan:
        return ColumnarEvidence(raws, luts, None, n, addrs)
    has_nan = np.zeros(len(columns), dtype=np.uint8)
    _scan_negative(addrs, n, has_nan)
    return ColumnarEvidence(raws, luts, _nan_groups(raws, has_nan, n), n)


# frame schemas already ingested: (model, epoch, columns, the columns' CategoricalDtype objects) -> their LUTs,
# when every category of every column is a state name.  A frame of the same schema (the same dtype objects:
# the same frame again, or frames built from one dtype per variable) then skips the per-column CPD and LUT
# lookups (a 1,038-column munin frame: ~0.5 ms of the ~2.2 ms predict_probability).  The dtype objects are
# kept referenced, so their ids stay theirs while cached.
_SCHEMA_CACHE = {}
_SCHEMA_CACHE_MAX = 32


def _schema_key(model, columns, dtypes):
    return (id(model), model.__dict__.get("_epoch", 0), tuple(columns), tuple(map(id, dtypes)))


def _schema_store(model, columns, cats, luts):
    dtypes = [a.dtype for a in cats]
    with _LUT_LOCK:
        if len(_SCHEMA_CACHE) >= _SCHEMA_CACHE_MAX:
            _SCHEMA_CACHE.clear()
        _SCHEMA_CACHE[_schema_key(model, columns, dtypes)] = (model, dtypes, list(luts))


def _schema_fast(model, columns, cats, n):
    """(raws, luts, addrs) of a frame whose schema was ingested before, or None (the general loop)."""
    dtypes = [a.dtype for a in cats]
    hit = _SCHEMA_CACHE.get(_schema_key(model, columns, dtypes))
    if hit is None or hit[0] is not model:
        return None
    try:
        raws = [a._codes for a in cats]
    except AttributeError:  # pragma: no cover - pandas internals moved
        return None
    i8 = np.dtype(np.int8)
    if not all(r.dtype is i8 and r.flags.c_contiguous for r in raws):
        return None
    if not n:
        return raws, hit[2], [0] * len(raws)
    addressof, char_at = ctypes.addressof, ctypes.c_char.from_buffer
    try:
        addrs = [addressof(char_at(r)) for r in raws]
    except (TypeError, ValueError):  # a read-only buffer: the general loop
        return None
    return raws, hit[2], addrs


def _scan_negative(addrs, n, has_nan):
    """has_nan[j] = 1 when column j (int8 category codes at addrs[j], n rows) holds a -1 (NaN):
    the native scan on _host_threads() threads."""
    nc = len(addrs)
    if nc and n:
        ptrs = (ctypes.c_void_p * nc)(*addrs)
        N.check(N.load_library().pgm_host_any_negative_i8(ptrs, nc, n, has_nan.ctypes.data_as(ctypes.c_void_p),
                                                          _host_threads()), "host_any_negative_i8")


def _nan_groups(raws, has_nan, n):
    """Rows grouped by their missing-column pattern, from the NaN-holding columns only."""
    nc = len(raws)
    nan_cols = np.nonzero(has_nan)[0].tolist()
    if not nan_cols or n == 0:
        groups = [(np.ones(nc, dtype=bool), np.arange(n))]
    else:
        miss = np.stack([raws[j] < 0 for j in nan_cols])  # [k, n]
        packed = np.packbits(miss.T, axis=1)
        _, first, inv = np.unique(packed, axis=0, return_index=True, return_inverse=True)
        inv = inv.reshape(-1)
        order = np.argsort(inv, kind="stable")
        bounds = np.searchsorted(inv[order], np.arange(len(first) + 1))
        groups = []
        for g in range(len(first)):
            rows = order[bounds[g]:bounds[g + 1]]
            mask = np.ones(nc, dtype=bool)
            for k, j in enumerate(nan_cols):
                if miss[k, rows[0]]:
                    mask[j] = False
            groups.append((mask, rows))
        groups.sort(key=lambda gr: gr[1][0])
    return groups


def _host_row_hash(codes):
    """[n, 2] int64 content hash of the rows of uint8 codes [n_cols, n] (host encoder path)."""
    rng = np.random.default_rng(_COL_KEY_SEED + 1)
    mult = rng.integers(1, 2 ** 63, size=(2, codes.shape[0]), dtype=np.int64) | 1
    h = np.zeros((codes.shape[1], 2), dtype=np.int64)
    with np.errstate(over="ignore"):
        for c in range(codes.shape[0]):
            x = codes[c].astype(np.int64) + 1
            h[:, 0] += x * mult[0, c]
            h[:, 1] ^= (x * mult[1, c]) >> 3
    return h


def upload_codes(codes):
    """Host uint8 [n_cols, n] -> device (through pgm_memcpy_h2d)."""
    import torch

    L = N.lib()
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    t = torch.empty(codes.shape, dtype=torch.uint8, device=E.device())
    if codes.size:
        N.check(L.pgm_memcpy_h2d(N.ptr(t), codes.ctypes.data_as(ctypes.c_void_p), codes.nbytes, N.stream_handle()),
                "memcpy_h2d")
    return t


def download(t):
    """Device tensor -> numpy through pgm_memcpy_d2h."""
    import torch

    L = N.lib()
    dt = {torch.float64: np.float64, torch.int32: np.int32, torch.int64: np.int64, torch.uint8: np.uint8}[t.dtype]
    if not t.is_contiguous():
        raise ValueError("download needs a contiguous tensor")
    out = np.empty(tuple(t.shape), dtype=dt)
    if out.size:
        N.check(L.pgm_memcpy_d2h(out.ctypes.data_as(ctypes.c_void_p), N.ptr(t), out.nbytes, N.stream_handle()),
                "memcpy_d2h")
    return out


def group_patterns(codes):
    """Rows grouped by which columns are observed: list of (observed column mask, row indices)."""
    miss = codes == MISSING  # [n_cols, n]
    if not miss.any():
        return [(np.ones(codes.shape[0], dtype=bool), np.arange(codes.shape[1]))]
    packed = np.packbits(miss.T, axis=1)
    uniq, inv = np.unique(packed, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    groups = []
    for g in range(len(uniq)):
        rows = np.nonzero(inv == g)[0]
        groups.append((~miss[:, rows[0]], rows))
    return groups


_PLAN_CACHE_ATTR = "_pgmpy_amd_plan_cache"
_PLAN_CACHE_MAX = 64
_plan_cache_lock = threading.Lock()


def get_plan(model, variables, evidence_vars, col_of, key=None):
    """The compiled plan of an evidence pattern, cached on the model (at most 64, least recently
    used dropped first).  A cached plan is reused only while PatternPlan.is_current(): the model's
    structure and the values of the CPDs it read are unchanged (a CPD edited, replaced, added or
    removed recompiles, as the reference recomputes from the current CPDs on every call)."""
    # evidence variable -> codes column, in evidence_vars order (one pass: munin patterns hold ~1,000);
    # `key`: the same tuple, precomputed by a caller that caches it per frame schema
    if key is None:
        key = (tuple(variables), tuple(evidence_vars), tuple(col_of.get(k, -1) for k in evidence_vars))
    with _plan_cache_lock:
        cache = model.__dict__.get(_PLAN_CACHE_ATTR)
        if cache is None:
            cache = model.__dict__.setdefault(_PLAN_CACHE_ATTR, {})
        plan = cache.pop(key, None)
        if plan is None or not plan.is_current():
            plan = PatternPlan(model, variables, evidence_vars, col_of)
            while len(cache) >= _PLAN_CACHE_MAX:
                cache.pop(next(iter(cache)))
        cache[key] = plan
    return plan


def _ingest(model, data, defer_scan=False):
    """(columns, col_of, evidence) of a frame: the zero-copy Categorical path when every column is
    one (its NaN scan left pending when defer_scan), else the general encoder."""
    columns = list(data.columns)
    col_of = {c: i for i, c in enumerate(columns)}
    ev = ingest_columnar(model, data, columns, defer_scan=defer_scan)
    if ev is None:
        ev = ingest_frame(model, data, columns)
    return columns, col_of, ev


def _direct_speculative(model, data, ingested, variables, marginals):
    """The direct path of a large categorical frame, overlapped with its NaN scan: while the scan runs on
    a worker thread, the plan of the all-observed pattern maps, uploads, runs and downloads (the scan and
    the device path take ~0.6 ms each on a 100 k-row munin frame).  Returns (plan, pinned result) when
    the scan then finds no NaN (the frame is that one pattern), else None — the result is discarded and
    the caller takes the grouped path with the groups the scan built.  An evidence code out of range raises
    only when the frame had no NaN (a NaN cell reaches the kernel as an out-of-range code)."""
    columns, col_of, ev = ingested
    if not isinstance(ev, ColumnarEvidence) or ev.groups is not None or len(data) < FAST_MIN_ROWS:
        return None
    ev.start_scan()
    plan, host, error = None, None, None
    try:
        plan = get_plan(model, list(variables), columns, col_of)
        if plan.kind == "fused" and list(plan.variables) == list(variables):
            host = _fused_to_host(plan, ev, columns, col_of, len(data), marginals)
    except IndexError as e:
        error = e
    finally:
        ev.finish_scan()
    if len(ev.groups) != 1 or not ev.groups[0][0].all():
        return None
    if error is not None:
        raise error
    return (plan, host) if host is not None else None


# frames of at least this many rows that are one evidence pattern of a fused plan take the direct path
# (_fused_to_host: pinned staging both ways, outputs handed to the result frame without a copy)
FAST_MIN_ROWS = int(os.environ.get("PGM_API_FAST_MIN_ROWS", 50_000))

# column structures of frames seen before: id(columns Index) -> (the Index, model, epoch, columns list,
# col_of, the plan-cache key part of col_of).  A pandas Index is immutable, so the same object means the
# same columns; the entry keeps it referenced, so its id stays its own while cached.
_FRAME_COLS = {}
_FRAME_COLS_MAX = 32
_SCAN_CHUNK = 128  # columns per native scan push while the frame is walked


_COLUMN_CHECKS = {}


def column_checks(model, data):
    """The reference's column checks of predict / predict_probability (DiscreteBayesianNetwork.py:
    850-856, 960-966: no variable missing, or a column that is not a node: ValueError) and the missing
    variables in its set order, cached per (columns Index object, model structure epoch): a 1,038-column
    frame builds four sets of ~1,000 names per call otherwise (~0.15 ms of a 1 ms predict_probability)."""
    cols = data.columns
    epoch = model.__dict__.get("_epoch", 0)
    hit = _COLUMN_CHECKS.get(id(cols))
    if hit is None or hit[0] is not cols or hit[1] is not model or hit[2] != epoch:
        nodes, have = set(model.nodes()), set(cols)
        status = "none" if have == nodes else ("extra" if have - nodes else "ok")
        hit = (cols, model, epoch, status, list(nodes - have))
        with _LUT_LOCK:
            if len(_COLUMN_CHECKS) >= _FRAME_COLS_MAX:
                _COLUMN_CHECKS.clear()
            _COLUMN_CHECKS[id(cols)] = hit
    if hit[3] == "none":
        raise ValueError("No variable missing in data. Nothing to predict")
    if hit[3] == "extra":
        raise ValueError("Data has variables which are not in the model")
    return list(hit[4])


_RESULT_COLS = {}


def _result_columns(model, order):
    """predict_probability's result columns f"{var}_{state}" (DiscreteBayesianNetwork.py:985-988) as a
    pandas Index, cached per (model structure epoch, missing variables)."""
    import pandas as pd

    key = (id(model), model.__dict__.get("_epoch", 0), tuple(order))
    hit = _RESULT_COLS.get(key)
    if hit is None or hit[0] is not model:
        names = pd.Index([var + "_" + str(s) for var in order for s in model.get_cpds(var).state_names[var]])
        if len(_RESULT_COLS) >= _FRAME_COLS_MAX:
            _RESULT_COLS.clear()
        hit = _RESULT_COLS[key] = (model, names)
    return hit[1]


def _frame_columns(model, data):
    cols = data.columns
    epoch = model.__dict__.get("_epoch", 0)
    hit = _FRAME_COLS.get(id(cols))
    if hit is not None and hit[0] is cols and hit[1] is model and hit[2] == epoch:
        return hit[3:]
    if cols.has_duplicates:
        return None
    columns = list(cols)
    node_map = getattr(model, "_node", None)
    if node_map is None or not all(c in node_map for c in columns):
        return None  # a column that is not a node: the general path raises the reference's error
    col_of = {c: i for i, c in enumerate(columns)}
    ent = (cols, model, epoch, columns, col_of, tuple(columns), tuple(range(len(columns))))
    with _LUT_LOCK:
        if len(_FRAME_COLS) >= _FRAME_COLS_MAX:
            _FRAME_COLS.clear()
        _FRAME_COLS[id(cols)] = ent
    return ent[3:]


def _direct_categorical(model, data, order, marginals):
    """The public API's direct path for a large pandas Categorical frame (r06), or None
    (the general path then runs, with the reference's errors).

    The device work of the all-observed pattern goes out FIRST: the plan's few evidence columns (7 of
    munin's 1,038) LUT-mapped on the host pool into pinned staging (pgm_host_lut_map_u8; a column whose
    categories are the state names in order is copied as is), uploaded, the fused pass launched, the
    result DMA'd into pinned memory, all asynchronous on the stream.  Then, while the GPU and the copy run,
    the frame is walked once in Python (each column's codes address and dtype) and the addresses are
    pushed, 128 columns at a time, to the native NaN scan (pgm_host_scan_begin / _push / _end) that runs
    on the host pool behind the walk.  A NaN anywhere (another evidence pattern) discards the result;
    otherwise the frame's schema is validated (every category a state name: the schema cache of
    _schema_fast, else _category_lut per column) and the result block is returned.  r05 did the walk,
    the scan and the mapping one after the other on the critical path (1.6 ms per 100 k rows)."""
    import torch

    n = len(data)
    if n < FAST_MIN_ROWS:
        return None
    fc = _frame_columns(model, data)
    if fc is None:
        return None
    columns, col_of, tcols, colidx = fc
    try:
        mgr = data._mgr
        arrays = mgr.arrays
        if len(arrays) != len(columns) or not np.array_equal(mgr.blknos, np.arange(len(columns))):
            return None
    except Exception:  # pandas internals moved: the general path
        return None
    cat_t = pd_categorical()
    L = N.lib()
    key = (tuple(order), tcols, colidx)
    plan = get_plan(model, list(order), columns, col_of, key=key)
    if plan.kind != "fused" or list(plan.variables) != list(order):
        return None
    used = [col_of[v] for v in plan.ev_used]
    srcs, luts = [], []
    for j in used:
        a = arrays[j]
        if type(a) is not cat_t:
            return None
        raw = a._codes
        if raw.dtype != np.int8 or not raw.flags.c_contiguous:
            return None
        st = model.get_cpds(columns[j]).state_names[columns[j]]
        lut, ok = _category_lut(columns[j], st, a.dtype)
        if not ok:
            return None  # a category that is not a state name: the general path raises for its cells
        srcs.append(raw)
        luts.append(None if _lut_is_identity(lut, len(a.dtype.categories)) else lut)
    s = N.stream_handle()
    k = max(1, len(used))
    stage = _pinned((k, n), torch.uint8)
    if used:
        sp = (ctypes.c_void_p * len(used))(*[r.ctypes.data for r in srcs])
        lp = (ctypes.c_void_p * len(used))(*[None if t is None else t.ctypes.data for t in luts])
        N.check(L.pgm_host_lut_map_u8(sp, lp, len(used), n, stage.ctypes.data_as(ctypes.c_void_p), n,
                                      _host_threads()), "host_lut_map_u8")
    dcodes = torch.empty(stage.shape, dtype=torch.uint8, device=E.device())
    N.check(L.pgm_memcpy_h2d(N.ptr(dcodes), stage.ctypes.data_as(ctypes.c_void_p), stage.nbytes, s), "memcpy_h2d")
    run_plan = plan.compact()
    out = run_plan.alloc_outputs(n, marginals=marginals, map_=not marginals)
    err = torch.zeros(1, dtype=torch.int32, device=dcodes.device)
    run_plan.run(dcodes, n, 0, n, out, err=err)
    dev = out["marg" if marginals else "map"]
    host = _pinned(tuple(dev.shape), dev.dtype)
    herr = _pinned((1,), torch.int32)
    N.check(L.pgm_memcpy_d2h_async(herr.ctypes.data_as(ctypes.c_void_p), N.ptr(err), 4, s), "memcpy_d2h")
    N.check(L.pgm_memcpy_d2h_async(host.ctypes.data_as(ctypes.c_void_p), N.ptr(dev), host.nbytes, s), "memcpy_d2h")
    # the walk + scan, overlapped with the GPU work and the copies queued above
    nc = len(columns)
    job = ctypes.c_void_p()
    N.check(L.pgm_host_scan_begin(n, nc, _host_threads(), ctypes.byref(job)), "host_scan_begin")
    ok = True
    dtypes = []
    addressof, char_at = ctypes.addressof, ctypes.c_char.from_buffer
    i8 = np.dtype(np.int8)
    try:
        for c0 in range(0, nc, _SCAN_CHUNK):
            part = arrays[c0:c0 + _SCAN_CHUNK]
            if not all(type(a) is cat_t for a in part):
                ok = False
                break
            raws = [a._codes for a in part]
            if not all(r.dtype is i8 and r.flags.c_contiguous for r in raws):
                ok = False
                break
            dtypes.extend([a.dtype for a in part])
            ptrs = (ctypes.c_void_p * len(raws))(*[addressof(char_at(r)) for r in raws])
            N.check(L.pgm_host_scan_push(job, ptrs, len(raws)), "host_scan_push")
    except (TypeError, ValueError):  # a read-only codes buffer: the general path
        ok = False
    finally:
        has_nan = np.zeros(nc, dtype=np.uint8)
        got = ctypes.c_int32()
        N.check(L.pgm_host_scan_end(job, has_nan.ctypes.data_as(ctypes.c_void_p), ctypes.byref(got)), "host_scan_end")
    N.check(L.pgm_stream_sync(s), "stream_sync")  # the staging / result buffers are released only after this
    if not ok or got.value != nc or has_nan.any():
        return None
    skey = _schema_key(model, columns, dtypes)
    hit = _SCHEMA_CACHE.get(skey)
    if hit is None or hit[0] is not model:
        all_luts = []
        for j, d in enumerate(dtypes):  # first frame of this schema: every category a state name?
            lut, lut_ok = _category_lut(columns[j], model.get_cpds(columns[j]).state_names[columns[j]], d)
            if not lut_ok:
                return None
            all_luts.append(lut)
        _schema_store(model, columns, arrays, all_luts)
    if herr[0] != 0:
        raise IndexError("evidence state code out of range")
    return plan, host


def pd_categorical():
    import pandas as pd

    return pd.Categorical


def _lut_is_identity(lut, n_cat):
    """The LUT maps category i to state i for every category (and NaN to MISSING): the codes can be
    used as they are."""
    return bool(lut[255] == MISSING and n_cat <= 127 and np.array_equal(lut[:n_cat], np.arange(n_cat)))


def _single_fused_plan(model, data, columns, col_of, ev, variables):
    """The fused plan when the whole frame is ONE evidence pattern with no NaN column (so the query
    variables are exactly `variables`, in order) and at least FAST_MIN_ROWS rows; else None."""
    if len(ev.groups) != 1 or len(data) < FAST_MIN_ROWS:
        return None
    mask, _ = ev.groups[0]
    if not mask.all():
        return None
    plan = get_plan(model, list(variables), columns, col_of)
    if plan.kind != "fused" or list(plan.variables) != list(variables):
        return None
    return plan


# result blocks above this many bytes are pinned with pgm_host_alloc instead of torch's caching host
# allocator: a result frame built on the block keeps it page-locked for as long as the
# caller keeps the frame, and torch's allocator would keep it cached (locked) after that as well, so
# repeated large predictions could exhaust the lockable memory; pgm_host_alloc memory is unlocked
# and returned when the last array on it is freed (a hipHostMalloc per call: ~0.1 ms per 100 MB)
PINNED_CACHE_MAX = int(os.environ.get("PGM_API_PINNED_CACHE_MAX", 64 << 20))


def _pinned(shape, dtype):
    """A page-locked host array that DMA reads / writes directly.  Small blocks come from torch's
    caching host allocator (their memory returns to its cache when the last array viewing it is
    freed); blocks above PINNED_CACHE_MAX bytes from pgm_host_alloc, released to the system when
    the last array viewing them (e.g. the result frame built on them) is freed."""
    import torch

    t = torch.empty(0, dtype=dtype)
    nbytes = int(np.prod(shape)) * t.element_size()
    if nbytes > PINNED_CACHE_MAX:
        return N.HostBuffer(tuple(shape), t.numpy().dtype).array
    return torch.empty(shape, dtype=dtype, pin_memory=True).numpy()


def _fused_to_host(plan, ev, columns, col_of, n, marginals):
    """The direct path of a one-pattern frame: the plan's evidence columns (LUT-mapped straight into a
    pinned staging buffer when the frame is categorical) uploaded, one launch of the fused pass, the
    outputs DMA'd into pinned host memory that the caller keeps (no further copy), one synchronize.
    Returns the marginals [n_acc, n] f64 or the MAP flat index [n] int32 (numpy, pinned)."""
    import torch

    L = N.lib()
    s = N.stream_handle()
    if isinstance(ev, ColumnarEvidence):
        used = [col_of[v] for v in plan.ev_used]
        stage = _pinned((max(1, len(used)), n), torch.uint8)
        for i, j in enumerate(used):
            np.take(ev.luts[j], ev.raws[j].view(np.uint8), out=stage[i])
        dcodes = torch.empty(stage.shape, dtype=torch.uint8, device=E.device())
        N.check(L.pgm_memcpy_h2d(N.ptr(dcodes), stage.ctypes.data_as(ctypes.c_void_p), stage.nbytes, s), "memcpy_h2d")
        run_plan = plan.compact()
    else:
        dcodes = ev.rows_codes(ev.groups[0][1])
        run_plan = plan
    out = run_plan.alloc_outputs(n, marginals=marginals, map_=not marginals)
    err = torch.zeros(1, dtype=torch.int32, device=dcodes.device)
    run_plan.run(dcodes, n, 0, n, out, err=err)
    key = "marg" if marginals else "map"
    dev = out[key]
    host = _pinned(tuple(dev.shape), dev.dtype)
    herr = _pinned((1,), torch.int32)
    N.check(L.pgm_memcpy_d2h_async(herr.ctypes.data_as(ctypes.c_void_p), N.ptr(err), 4, s), "memcpy_d2h")
    N.check(L.pgm_memcpy_d2h(host.ctypes.data_as(ctypes.c_void_p), N.ptr(dev), host.nbytes, s), "memcpy_d2h")
    if herr[0] != 0:
        raise IndexError("evidence state code out of range")
    return host


def _run_groups(model, data, base_vars, want_marg, want_map, extra_nan_vars, ingested=None):
    """Yield (plan, rows, outputs-on-host) per evidence pattern."""
    columns, col_of, ev = ingested if ingested is not None else _ingest(model, data)
    for mask, rows in ev.groups:
        observed = [columns[j] for j in range(len(columns)) if mask[j]]
        nan_cols = [columns[j] for j in range(len(columns)) if not mask[j]]
        variables = list(base_vars) + ([c for c in nan_cols if c not in base_vars] if extra_nan_vars else [])
        plan = get_plan(model, variables, observed, col_of)
        if isinstance(ev, ColumnarEvidence):  # only the columns this pattern's plan reads
            dcodes = ev.codes_for([col_of[v] for v in plan.ev_used], rows)
            plan = plan.compact()
        else:
            dcodes = ev.rows_codes(rows)
        n = len(rows)
        out = plan.alloc_outputs(n, marginals=want_marg, map_=want_map)
        err = None
        import torch

        err = torch.zeros(1, dtype=torch.int32, device=dcodes.device)
        plan.run(dcodes, n, 0, n, out, err=err)
        if int(download(err)[0]) != 0:
            raise IndexError("evidence state code out of range")
        host = {k: download(v) for k, v in out.items()}
        yield plan, rows, host



def wide_columns(model, columns):
    """Evidence columns whose variable has more states than the uint8 codes of the batched plans hold
    (state numbers 0..253; 254 marks a non-state, 255 = NaN).  The reference has no such limit
    (utils/state_name.py:71-84): frames with one of these take _rowwise_frame.  The model's largest
    state count is cached per structure epoch (a 1,038-column munin frame: one check, not 1,038
    get_cardinality calls, ~0.6 ms)."""
    cpds = model.get_cpds()
    key = (model.__dict__.get("_epoch", 0), len(cpds))
    hit = model.__dict__.get("_pgmpy_amd_max_card")
    if hit is None or hit[0] != key:
        hit = model.__dict__["_pgmpy_amd_max_card"] = (key, max((int(c.cardinality[0]) for c in cpds), default=0))
    if hit[1] < MISSING:
        return []
    return [c for c in columns if int(model.get_cardinality(c)) >= MISSING]


def _rowwise_frame(model, data, kind, seed=None):
    """predict / predict_probability / query_batch for frames with a wide evidence column (see
    wide_columns): the reference's own loop over distinct rows (DiscreteBayesianNetwork.py:866-910:
    groupby over every column with dropna=False, one query per distinct row), each query a device
    VariableElimination call (the strided-view contraction path, which takes any state count).  NaN
    cells are unobserved, as in the batched path.  kind: "marg" (predict_probability), "map"
    (predict), "sample" (predict(stochastic=True): DiscreteFactor.sample of the row's joint with a
    fresh Generator(seed) per distinct row, L879-882)."""
    import pandas as pd

    from .ExactInference import VariableElimination

    columns = list(data.columns)
    order = list(set(model.nodes()) - set(columns))
    n = len(data)
    ve = VariableElimination(model)
    groups = data.groupby(columns, dropna=False, sort=False).indices if n else {}
    if kind == "marg":
        cols = {var + "_" + str(s): np.empty(n) for var in order for s in model.get_cpds(var).state_names[var]}
    else:
        vals = {c: np.full(n, np.nan, dtype=object) for c in order}
        filled = {}
    for key, rows in groups.items():
        key = key if isinstance(key, tuple) else (key,)
        evidence = {c: v for c, v in zip(columns, key) if not pd.isna(v)}
        if kind == "marg":
            res = ve.query(order, evidence, joint=False, show_progress=False)
            for var in order:
                for k, st in enumerate(model.get_cpds(var).state_names[var]):
                    cols[var + "_" + str(st)][rows] = float(np.asarray(res[var].values)[k])
            continue
        variables = order + [c for c in columns if c not in evidence]
        if kind == "map":
            assignment = ve.map_query(variables, evidence, show_progress=False)
            draws = {v: np.full(len(rows), assignment[v], dtype=object) for v in variables}
        else:
            smp = ve.query(variables, evidence, joint=True, show_progress=False).sample(len(rows), seed=seed)
            draws = {v: smp[v].to_numpy(object) for v in variables}
        for v in variables:
            if v in vals:
                vals[v][rows] = draws[v]
            else:
                if v not in filled:
                    filled[v] = data[v].to_numpy(object).copy()
                filled[v][rows] = draws[v]
    if kind == "marg":
        return pd.DataFrame(cols, index=data.index)
    base = data.assign(**filled) if filled else data
    out = pd.concat([base, pd.DataFrame(vals, index=data.index, columns=order)], axis=1)
    return out if out.index.is_monotonic_increasing else out.sort_index()


def predict_probability_frame(model, data):
    """DiscreteBayesianNetwork.predict_probability (DiscreteBayesianNetwork.py:912-989)."""
    import pandas as pd

    order = column_checks(model, data)  # the reference's set iteration order (column order of its output)
    n = len(data)
    if n == 0:  # the reference builds its frame from empty per-column lists: no columns at all
        return pd.DataFrame({}, index=data.index)
    if wide_columns(model, data.columns):
        return _rowwise_frame(model, data, "marg")
    direct = _direct_categorical(model, data, order, True)
    marg = direct[1] if direct is not None else None
    if marg is None:
        ingested = _ingest(model, data, defer_scan=n >= FAST_MIN_ROWS)
        direct = _direct_speculative(model, data, ingested, order, True)
        marg = direct[1] if direct is not None else None
    if marg is None:
        if isinstance(ingested[2], ColumnarEvidence):
            ingested[2].finish_scan()
        plan = _single_fused_plan(model, data, *ingested, order)
        if plan is not None:
            marg = _fused_to_host(plan, ingested[2], ingested[0], ingested[1], n, True)
    if marg is not None:
        # one pattern: the marginals' rows ARE the result's columns (plan.variables == order, each
        # variable's states consecutive), so the frame is built on the pinned output block, no copy
        names = _result_columns(model, order)
        assert len(names) == marg.shape[0]
        return pd.DataFrame(marg.T, columns=names, index=data.index, copy=False)
    cols = {}
    for var in order:
        for s in model.get_cpds(var).state_names[var]:
            cols[var + "_" + str(s)] = np.empty(n)
    for plan, rows, host in _run_groups(model, data, order, True, False, False, ingested):
        for i, var in enumerate(plan.variables[:len(order)]):
            a = plan.acc_off[i]
            for k, s in enumerate(plan.states[var]):
                cols[var + "_" + str(s)][rows] = host["marg"][a + k]
    return pd.DataFrame(cols, index=data.index)


def _append_columns(base, vals, order):
    """base's columns then vals[c] for c in order, as a new frame whose observed columns share base's
    buffers (as DataFrame.copy(deep=False) shares them; DESIGN.md deviation 5).  Default: one new
    BlockManager holding base's blocks plus one block per new column (a munin frame has ~1,000
    categorical blocks: setting columns one by one on a copy costs ~2 ms each, pd.concat copies
    every block).  PGM_API_APPEND=concat (A/B): pd.concat of the two frames (independent copies);
    =shallow: a shallow copy with the columns set on it.  Any pandas-internals mismatch falls back
    to the shallow form."""
    import warnings

    import pandas as pd

    mode = os.environ.get("PGM_API_APPEND", "blocks")
    if mode == "concat":
        return pd.concat([base, pd.DataFrame(vals, index=base.index, columns=order)], axis=1)
    if mode == "blocks":
        try:
            from pandas._libs.internals import BlockPlacement
            from pandas.core.internals.blocks import new_block
            from pandas.core.internals.managers import BlockManager

            nb = len(base.columns)
            blocks = list(base._mgr.blocks)
            for k, c in enumerate(order):
                v = np.asarray(vals[c])
                blocks.append(new_block(v.reshape(1, -1), placement=BlockPlacement(slice(nb + k, nb + k + 1)),
                                        ndim=2))
            axes = [base.columns.append(pd.Index(list(order))), base.index]
            return pd.DataFrame._from_mgr(BlockManager(tuple(blocks), axes, verify_integrity=False), axes=axes)
        except Exception:  # pragma: no cover - pandas internals moved: the public form below
            pass
    out = base.copy(deep=False)
    with warnings.catch_warnings():  # a frame of ~1,000 categorical blocks is "fragmented" by design
        warnings.simplefilter("ignore", pd.errors.PerformanceWarning)
        for c in order:
            out[c] = vals[c]
    return out


def predict_frame(model, data):
    """DiscreteBayesianNetwork.predict, MAP (DiscreteBayesianNetwork.py:731-910)."""
    import pandas as pd

    order = column_checks(model, data)
    if len(data) == 0:  # the reference indexes the first group of an empty groupby
        raise IndexError("list index out of range (predict on an empty DataFrame)")
    if wide_columns(model, data.columns):
        return _rowwise_frame(model, data, "map")
    direct = _direct_categorical(model, data, order, False)
    ingested = None
    if direct is None:
        ingested = _ingest(model, data, defer_scan=len(data) >= FAST_MIN_ROWS)
        direct = _direct_speculative(model, data, ingested, order, False)
    if direct is None:
        if isinstance(ingested[2], ColumnarEvidence):
            ingested[2].finish_scan()
        plan = _single_fused_plan(model, data, *ingested, order)
        if plan is not None:
            direct = plan, _fused_to_host(plan, ingested[2], ingested[0], ingested[1], len(data), False)
    if direct is not None:  # one pattern, no NaN cell: the MAP columns straight from the pinned index
        plan = direct[0]
        idx = direct[1].astype(np.int64)
        vals = {}
        for i in reversed(range(len(plan.variables))):
            var, c = plan.variables[i], plan.cards[i]
            vals[var] = np.array(plan.states[var], dtype=object)[idx % c]
            idx //= c
        out = _append_columns(data, vals, order)
        return out if out.index.is_monotonic_increasing else out.sort_index()
    vals = {c: np.full(len(data), np.nan, dtype=object) for c in order}
    # the observed columns keep their dtype (object frames stay object, as the reference's merge
    # leaves them; a categorical frame is not expanded to 10^8 Python objects)
    base = data
    filled = {}  # observed columns whose NaN cells receive MAP states, as in the reference
    for plan, rows, host in _run_groups(model, data, order, False, True, True, ingested):
        idx = host["map"].astype(np.int64)
        # decode the flat index (C-order over plan.variables, last fastest)
        for i in reversed(range(len(plan.variables))):
            var = plan.variables[i]
            c = plan.cards[i]
            st = np.array(plan.states[var], dtype=object)
            if var in vals:
                vals[var][rows] = st[idx % c]
            else:
                if var not in filled:
                    filled[var] = base[var].to_numpy(object).copy()
                filled[var][rows] = st[idx % c]
            idx = idx // c
    if filled:
        base = base.assign(**filled)  # a new frame: the caller's data is not modified
    # the observed columns (object, as the reference's merge leaves them), then the MAP columns in the
    # reference's set order, rows sorted by index (DiscreteBayesianNetwork.py:895-910)
    out = _append_columns(base, vals, order)
    if out.index.is_monotonic_increasing:
        return out
    return out.sort_index()


def _hash_groups_exact(ev, first, inv):
    """Every row's codes equal its hash group's representative row (no 128-bit collision merged two
    different evidence rows): one device comparison of the codes against the representatives."""
    import torch

    if len(first) == ev.n:
        return True
    idx = torch.as_tensor(first[inv].astype(np.int64), device=ev.codes.device)
    return bool(torch.equal(ev.codes.index_select(1, idx), ev.codes))


def _raw_values_ambiguous(model, data, columns, fallback_cols=None):
    """Whether two distinct raw cell values of a column map to one state (the str() fallback:
    1 and "1"; or two categories with the same state), so grouping by state codes would merge rows
    the reference's groupby over raw values keeps apart.  fallback_cols: the columns ingestion saw
    use the str() fallback (only those can be ambiguous); None = check every column."""
    import pandas as pd

    states = model.states
    for col in columns:
        if fallback_cols is not None and col not in fallback_cols:
            continue
        v = data[col]
        st = list(states[col])
        if isinstance(v.dtype, pd.CategoricalDtype):
            v = pd.Series(v.cat.categories)
        if v.dtype != object:
            continue  # one numeric/bool dtype: str() is one to one on it
        vals = v.dropna().to_numpy(dtype=object)
        if len(vals) and (_lookup_codes(vals, st) < 0).any():
            return True  # some cell reaches its state through str(): mixed raw types may merge
    return False


def predict_stochastic_frame(model, data, seed=None):
    """DiscreteBayesianNetwork.predict(stochastic=True) (DiscreteBayesianNetwork.py:866-910).

    The reference de-duplicates identical rows (groupby over every column, L867-870), queries the
    joint of the missing variables (plus the row's NaN columns) once per unique row, and draws
    len(group) samples from it with a fresh numpy Generator(seed) per group (DiscreteFactor.sample,
    L868-912: Generator.choice = inverse CDF of fresh uniforms).  Here: rows are keyed by a 128-bit
    content hash computed in the ingestion pass, one joint per unique row comes from the pattern's
    compiled plan, and pgm_sample_joint inverts each row's CDF on the device with the uniform the
    reference's stream gives that row (its position in its group)."""
    import pandas as pd
    import torch

    columns = list(data.columns)
    col_of = {c: i for i, c in enumerate(columns)}
    missing_variables = set(model.nodes()) - set(data.columns)
    order = list(missing_variables)
    n = len(data)
    if n == 0:
        raise IndexError("list index out of range (predict on an empty DataFrame)")
    if wide_columns(model, columns):
        return _rowwise_frame(model, data, "sample", seed=seed)
    ev = ingest_frame(model, data, columns, row_hash=True)
    _, first, inv = np.unique(ev.row_hash, axis=0, return_index=True, return_inverse=True)
    inv = inv.reshape(-1)
    if not _hash_groups_exact(ev, first, inv) or \
            _raw_values_ambiguous(model, data, columns, getattr(ev, "fallback_cols", None)):
        # a hash collision, or cells whose raw values differ but reach the same state (1 and "1"
        # through the str() fallback): the reference's own grouping of the raw values (L867)
        gid = data.groupby(columns, dropna=False, sort=False).ngroup().to_numpy()
        _, first, inv = np.unique(gid, return_index=True, return_inverse=True)
        inv = inv.reshape(-1)
    counts = np.bincount(inv, minlength=len(first))
    srt = np.argsort(inv, kind="stable")
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    pos = np.empty(n, dtype=np.int64)
    pos[srt] = np.arange(n) - np.repeat(starts, counts)
    if seed is None:  # a fresh entropy-seeded Generator per group: independent uniforms
        u = np.random.default_rng().random(n)
    else:  # every group restarts Generator(seed): a row's uniform is the stream at its position
        u = np.random.default_rng(seed).random(int(counts.max()) if n else 0)[pos]
    vals = {c: np.full(n, np.nan, dtype=object) for c in order}
    filled = {}
    L = N.lib()
    s = N.stream_handle()
    for mask, rows in ev.groups:
        observed = [columns[j] for j in range(len(columns)) if mask[j]]
        nan_cols = [columns[j] for j in range(len(columns)) if not mask[j]]
        variables = list(missing_variables.union(set(nan_cols)))  # the reference's query variables (L873-875)
        plan = get_plan(model, variables, observed, col_of)
        uniq = np.unique(inv[rows])
        reps = first[uniq]
        n_u = len(uniq)
        out = plan.alloc_outputs(n_u, marginals=False, joint=True)
        err = torch.zeros(1, dtype=torch.int32, device=ev.codes.device)
        plan.run(ev.rows_codes(reps), n_u, 0, n_u, out, err=err)
        if int(download(err)[0]) != 0:
            raise IndexError("evidence state code out of range")
        joint = out["joint"]  # [P, n_u], C-order over plan.variables
        if np.isnan(float(E.to_host(E.contract(joint, ["q", E.ROW], None, None, [], reduce="sum", combine="copy")))):
            raise ValueError("probabilities contain NaN")  # Generator.choice on an impossible row's joint
        grp = E.to_device_raw(np.searchsorted(uniq, inv[rows]).astype(np.int32))
        d_u = E.to_device_raw(np.ascontiguousarray(u[rows]))
        d_idx = torch.empty(len(rows), dtype=torch.int32, device=joint.device)
        N.check(L.pgm_sample_joint(N.ptr(joint), int(joint.stride(0)), int(plan.P), N.ptr(grp), N.ptr(d_u),
                                   len(rows), N.ptr(d_idx), s), "sample_joint")
        idx = download(d_idx).astype(np.int64)
        for i in reversed(range(len(plan.variables))):
            var = plan.variables[i]
            c = plan.cards[i]
            st = np.array(plan.states[var], dtype=object)
            if var in vals:
                vals[var][rows] = st[idx % c]
            else:
                if var not in filled:
                    filled[var] = data[var].to_numpy(object).copy()
                filled[var][rows] = st[idx % c]
            idx = idx // c
    base = data.assign(**filled) if filled else data
    out = pd.concat([base, pd.DataFrame(vals, index=data.index, columns=order)], axis=1)
    return out if out.index.is_monotonic_increasing else out.sort_index()


def query_batch(model, variables, evidence, joint=False):
    """P(variables | row) for every row of the evidence DataFrame (NaN = unobserved)."""
    n = len(evidence)
    res = None
    cards = [int(model.get_cardinality(v)) for v in variables]
    if joint:
        res = np.empty([n] + cards)
    else:
        res = {v: np.empty((n, c)) for v, c in zip(variables, cards)}
    columns = list(evidence.columns)
    col_of = {c: i for i, c in enumerate(columns)}
    if wide_columns(model, columns):  # per row through device VariableElimination (see _rowwise_frame)
        from .ExactInference import VariableElimination

        import pandas as pd

        ve = VariableElimination(model)
        for r in range(n):
            row = evidence.iloc[r]
            ev_r = {c: row[c] for c in columns if not pd.isna(row[c])}
            q = ve.query(list(variables), ev_r, joint=joint, show_progress=False)
            if joint:
                res[r] = np.asarray(q.values).transpose([q.variables.index(v) for v in variables])
            else:
                for v in variables:
                    res[v][r] = np.asarray(q[v].values)
        return res
    ev = ingest_frame(model, evidence, columns)
    import torch

    for mask, rows in ev.groups:
        observed = [columns[j] for j in range(len(columns)) if mask[j]]
        plan = get_plan(model, list(variables), observed, col_of)
        dcodes = ev.rows_codes(rows)
        m = len(rows)
        out = plan.alloc_outputs(m, marginals=not joint, joint=joint)
        err = torch.zeros(1, dtype=torch.int32, device=dcodes.device)
        plan.run(dcodes, m, 0, m, out, err=err)
        if int(download(err)[0]) != 0:
            raise IndexError("evidence state code out of range")
        if joint:
            j = download(out["joint"])  # [P, m]
            res[rows] = j.T.reshape([m] + cards)
        else:
            mg = download(out["marg"])
            for i, v in enumerate(variables):
                a = plan.acc_off[i]
                res[v][rows] = mg[a:a + cards[i]].T
    return res
