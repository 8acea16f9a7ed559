"""Evidence-pattern plan compiler for batched inference.

For one evidence *pattern* — the set of observed variables E and the query
variables Q — everything that does not depend on the observed *states* is
done once on the host:

  1. prune the network (d-separation + ancestral graph, pgmpy/inference/base.py:154-212),
     summing pruned parents out of CPDs on the device (TabularCPD.marginalize);
  2. drop factors whose scope is all evidence (ExactInference.py:383);
  3. pick an executor:
     * FUSED  (pgm_rows_plan_*): when the query+hidden index space is small, one
       kernel runs reduce -> sum-product -> normalize -> marginals / joint / MAP
       for every row, one lane per row, CPTs staged in LDS (the munin predict
       template of SURVEY.md §8(d) C3: 5 CPTs, 7 evidence columns, 180-entry joint);
     * STEPS: otherwise, per-row evidence gathers (pgm_gather) and a greedy
       pairwise path of fused product+marginalize kernels over tensors that
       carry an evidence-row axis (pgmpy_amd.inference.contraction).

Per batch only the uint8 evidence-code columns the plan reads are touched.
A compiled plan is immutable; run() is re-entrant on distinct outputs.
"""
import ctypes
import os
import threading
from operator import itemgetter

import numpy as np

from .. import _native as N
from .. import engine as E
from .base import prune_structure
from .contraction import contract_factors, plan_stats

FUSED_MAX_SPACE = 4096  # query x hidden index space per row for the fused kernel


def _values_epoch():
    """factors.discrete.DiscreteFactor.values_epoch, imported once (is_current runs on every single query)."""
    global _values_epoch
    from ..factors.discrete.DiscreteFactor import values_epoch

    _values_epoch = values_epoch
    return values_epoch()


class PatternPlan:
    """Compiled plan for (query variables, observed variables) on a DiscreteBayesianNetwork."""

    def __init__(self, model, variables, evidence_vars, col_of, force=None):
        self.model = model
        self.variables = list(variables)
        self.evidence_vars = list(evidence_vars)
        self.col_of = dict(col_of)
        overlap = set(self.variables) & set(self.evidence_vars)
        if overlap:
            raise ValueError(f"Can't have the same variables in both `variables` and `evidence`. "
                             f"Found in both: {overlap}")
        if not self.variables:
            raise ValueError("The `variables` argument to query() must contain at least one variable.")
        states = model.states
        self.states = {v: list(states[v]) for v in self.variables}
        self.cards = [len(self.states[v]) for v in self.variables]
        self.n_acc = int(sum(self.cards))
        self.acc_off = list(np.cumsum([0] + self.cards[:-1]))
        self.P = int(np.prod(self.cards))

        kept, ev = prune_structure(model, self.variables, self.evidence_vars)
        kept_set, ev_set = set(kept), set(ev)
        self._lock = threading.RLock()  # lazy compilation and shared scratch buffers
        self._epoch = getattr(model, "_epoch", None)
        self._sources = []  # (cpd, value token) of every CPD the plan read: see is_current()
        factors = []  # (vars, host values C-order)
        for var in kept:
            cpd = model.get_cpds(var)
            self._sources.append((cpd, cpd._value_token()))
            scope_diff = set(cpd.scope()) - kept_set
            if scope_diff:
                cpd = cpd.marginalize(scope_diff, inplace=False)  # device op
            vars_ = list(cpd.variables)
            if all(v in ev_set for v in vars_):
                continue  # ExactInference.py:383
            factors.append((vars_, cpd))
        self.factors = factors
        self.ev_used = sorted({v for vars_, _ in factors for v in vars_ if v in ev_set},
                              key=lambda v: self.col_of[v])
        hidden = []
        for vars_, _ in factors:
            for v in vars_:
                if v not in ev_set and v not in self.variables and v not in hidden:
                    hidden.append(v)
        self.hidden = hidden
        card = {v: int(model.get_cardinality(v)) for v in set(self.variables) | set(hidden) | ev_set}
        self.card = card
        self.H = int(np.prod([card[v] for v in hidden])) if hidden else 1
        n_ev_terms = sum(1 for vars_, _ in factors for v in vars_ if v in ev_set)
        comps = self.components()
        comp_space = max((int(np.prod([card[v] for v in q + h])) for q, h, _ in comps), default=1)
        fused_ok = (len(factors) <= N.ROWS_MAX_FAC and len(self.variables) + len(hidden) <= N.ROWS_MAX_LOOP
                    and n_ev_terms <= N.ROWS_MAX_EV and self.n_acc <= N.ROWS_MAX_MARG
                    and len(comps) <= N.ROWS_MAX_COMP and comp_space <= FUSED_MAX_SPACE)
        self.joint_fused_ok = fused_ok and self.P * self.H <= FUSED_MAX_SPACE
        self.kind = force or ("fused" if fused_ok else "steps")
        if self.kind == "fused" and not fused_ok:
            raise ValueError("pattern does not fit the fused row kernel")
        self._handle = None
        self._handle_joint = None
        self.extra_mode = 0  # tuning bits (N.ROWS_VALUES_GLOBAL)
        self.n_comp = len(comps) if self.kind == "fused" else None

    def is_current(self):
        """True while the model structure and the values of every CPD this plan read are unchanged
        (the reference recomputes from the current CPDs on every call)."""
        if getattr(self.model, "_epoch", None) != self._epoch:
            return False
        ve = _values_epoch()
        if ve == self.__dict__.get("_vepoch"):
            # no factor's values were replaced or newly handed out since the last full check: only
            # the exposed sources (host arrays a caller may edit in place) need their CRC compared
            return all(cpd._value_token() == tok for cpd, tok in self._exposed_sources)
        if not all(cpd._value_token() == tok for cpd, tok in self._sources):
            return False
        self._vepoch = ve
        self._exposed_sources = [(cpd, tok) for cpd, tok in self._sources if cpd._exposed]
        return True

    # ------------------------------------------------------------------ fused
    def components(self):
        """Independent components of the evidence-reduced factor graph over query + hidden vars.

        Returns [(query vars (original order), hidden vars, factor indices)], ordered by first query var."""
        loop = self.variables + self.hidden
        parent = {v: v for v in loop}

        def find(v):
            while parent[v] != v:
                parent[v] = parent[parent[v]]
                v = parent[v]
            return v

        for vars_, _ in self.factors:
            lv = [v for v in vars_ if v in parent]
            for v in lv[1:]:
                a, b = find(lv[0]), find(v)
                if a != b:
                    parent[b] = a
        groups = {}
        for v in loop:
            groups.setdefault(find(v), []).append(v)
        comps = []
        for root, members in groups.items():
            ms = set(members)
            q = [v for v in self.variables if v in ms]
            h = [v for v in self.hidden if v in ms]
            f = [i for i, (vars_, _) in enumerate(self.factors) if any(v in ms for v in vars_)]
            comps.append((q, h, f))
        order = {v: i for i, v in enumerate(loop)}
        comps.sort(key=lambda c: min(order[v] for v in c[0] + c[1]))
        return comps

    def kernel_name(self):
        """The device kernel pgm_rows_plan_run launches for this plan's marginal/MAP outputs: the
        plan-specialised hipRTC kernel `pgm_rows_jit` when every component has one query variable and
        no hidden variable (pgmhip.hip rows_jit_source; if hipRTC is unavailable the AOT
        k_rows_affine / k_rows run instead), else the table-driven k_rows."""
        if self.kind != "fused":
            return None
        for q, h, f in self.components():
            if len(q) != 1 or h:
                return "k_rows"
        return "pgm_rows_jit"

    def _rows_plan_struct(self, split):
        """(pgm_rows_plan, packed CPT values, component count): host-only."""
        comps = self.components() if split else [(list(self.variables), list(self.hidden),
                                                  list(range(len(self.factors))))]
        if len(comps) > N.ROWS_MAX_COMP:
            raise ValueError("too many independent components for the fused kernel")
        pl = N.RowsPlan()
        loop, fac_order = [], []
        for ci, (q, h, f) in enumerate(comps):
            pl.comp_loop_begin[ci] = len(loop)
            pl.comp_n_query[ci] = len(q)
            loop.extend(q + h)
            pl.comp_loop_end[ci] = len(loop)
            pl.comp_fac_begin[ci] = len(fac_order)
            fac_order.extend(f)
            pl.comp_fac_end[ci] = len(fac_order)
        pl.n_comp = len(comps)
        pl.n_loop = len(loop)
        pl.n_query = len(self.variables)
        pl.n_fac = len(fac_order)
        pl.n_marg = self.n_acc
        pl.n_joint = self.P
        map_stride = {v: int(np.prod(self.cards[i + 1:])) for i, v in enumerate(self.variables)}
        for i, v in enumerate(loop):
            pl.loop_card[i] = self.card[v]
            if v in self.variables:
                pl.loop_marg_off[i] = self.acc_off[self.variables.index(v)]
                pl.loop_map_stride[i] = map_stride[v]
            else:
                pl.loop_marg_off[i] = -1
                pl.loop_map_stride[i] = 0
        chunks, base, ev_terms = [], 0, []
        for f, fi in enumerate(fac_order):
            vars_, cpd = self.factors[fi]
            vals = self._host_values(fi)
            cards = [int(c) for c in cpd.cardinality]
            strides = [int(np.prod(cards[i + 1:])) for i in range(len(cards))]
            pl.fac_base[f] = base
            pl.fac_ev_begin[f] = len(ev_terms)
            for v, st in zip(vars_, strides):
                if v in loop:
                    pl.fac_stride[f][loop.index(v)] = st
                else:
                    ev_terms.append((self.col_of[v], st, self.card[v]))
            pl.fac_ev_end[f] = len(ev_terms)
            chunks.append(vals)
            base += vals.size
        pl.n_ev = len(ev_terms)
        for j, (col, st, c) in enumerate(ev_terms):
            pl.ev_col[j], pl.ev_stride[j], pl.ev_card[j] = col, st, c
        values = np.concatenate(chunks) if chunks else np.zeros(1)
        if values.size >= 2 ** 31:
            raise ValueError("plan values too large")
        pl.n_values = int(values.size)
        return pl, values, len(comps)

    def specialised_source(self):
        """Source of the plan-specialised (hipRTC) row kernel for this plan (pgm_rows_plan_source);
        host-only, no device needed."""
        pl, _, _ = self._rows_plan_struct(split=True)
        L = N.load_library()
        need = ctypes.c_size_t()
        N.check(L.pgm_rows_plan_source(ctypes.byref(pl), None, 0, ctypes.byref(need)), "rows_plan_source")
        buf = ctypes.create_string_buffer(need.value)
        N.check(L.pgm_rows_plan_source(ctypes.byref(pl), buf, need.value, None), "rows_plan_source")
        return buf.value.decode()

    def _make_rows_plan(self, split):
        pl, values, n_comp = self._rows_plan_struct(split)
        L = N.lib()
        h = ctypes.c_void_p()
        N.check(L.pgm_rows_plan_create(ctypes.byref(pl), values.ctypes.data_as(ctypes.c_void_p), ctypes.byref(h)),
                "rows_plan_create")
        return h, pl, n_comp

    def _host_values(self, fi):
        """CPT values (C-order) of factor fi, packed into the plan (a copy, no arithmetic)."""
        cache = self.__dict__.setdefault("_vals_cache", {})
        if fi not in cache:
            cache[fi] = np.ascontiguousarray(self.factors[fi][1]._values_readonly(), dtype=np.float64).reshape(-1)
        return cache[fi]

    def _build_fused(self):
        """Upload the plan (lazily, on first run)."""
        if self._handle is None:
            with self._lock:
                if self._handle is None:
                    h, self._plan, self.n_comp = self._make_rows_plan(split=True)
                    if self.n_comp == 1:
                        self._handle_joint = h
                    self._handle = h

    def shard_run(self, codes, devices, marginals=True, map_=False, out=None):
        """This fused plan over host rows sharded across GPUs through the C-ABI (pgm_rows_shard_run):
        codes = host uint8 [columns, n_rows] in this plan's column numbering (col_of), devices = the
        HIP device of each shard (contiguous row blocks, shard i on devices[i]; one plan handle per
        shard, created on its device and cached).  Returns {"marg": [n_acc, n_rows] f64, "map": [n_rows]
        int32} as numpy arrays, equal to run() over all rows.  out: the caller's arrays to write instead
        (same keys; pinned ones, e.g. pgmpy_amd._native.HostBuffer arrays, take the overlapped DMA path).
        The native path a non-Python caller uses (include/pgmhip.h); pgmpy_amd.distributed shards over
        processes instead."""
        if self.kind != "fused":
            raise ValueError("shard_run(): fused plans only")
        if not (isinstance(codes, np.ndarray) and codes.dtype == np.uint8 and codes.flags.c_contiguous):
            codes = np.ascontiguousarray(codes, dtype=np.uint8)
        n_cols, n_rows = codes.shape
        L = N.lib()
        cache = self.__dict__.setdefault("_shard_handles", {})
        handles = []
        for i, d in enumerate(devices):
            key = (i, int(d))
            if key not in cache:
                N.check(L.pgm_set_device(int(d)), "set_device")
                try:
                    cache[key] = self._make_rows_plan(split=True)[0]
                finally:
                    N.check(L.pgm_set_device(E.device().index or 0), "set_device")
            handles.append(cache[key])
        mode = (N.ROWS_MARGINALS if marginals else 0) | (N.ROWS_MAP if map_ else 0)
        out = out or {}
        marg = out.get("marg") if marginals else None
        mp = out.get("map") if map_ else None
        if marg is None and marginals:
            marg = np.empty((self.n_acc, n_rows), dtype=np.float64)
        if mp is None and map_:
            mp = np.empty(n_rows, dtype=np.int32)
        if marg is not None and (marg.dtype != np.float64 or marg.shape != (self.n_acc, n_rows)
                                 or not marg.flags.c_contiguous):
            raise ValueError(f"out['marg'] must be a C-contiguous float64 [{self.n_acc}, {n_rows}] array")
        if mp is not None and (mp.dtype != np.int32 or mp.shape != (n_rows,)):
            raise ValueError(f"out['map'] must be an int32 [{n_rows}] array")
        err = np.zeros(1, dtype=np.int32)
        arr = (ctypes.c_void_p * len(handles))(*[h.value for h in handles])
        N.check(L.pgm_rows_shard_run(arr, len(handles), mode, codes.ctypes.data_as(ctypes.c_void_p), n_rows, n_cols,
                                     n_rows, None if marg is None else marg.ctypes.data_as(ctypes.c_void_p), n_rows,
                                     None if mp is None else mp.ctypes.data_as(ctypes.c_void_p),
                                     err.ctypes.data_as(ctypes.c_void_p)), "rows_shard_run")
        if err[0]:
            raise IndexError("evidence state code out of range")
        return {"marg": marg, "map": mp}

    def _joint_handle(self):
        if self._handle_joint is None:
            with self._lock:
                if self._handle_joint is None:
                    self._handle_joint, _, _ = self._make_rows_plan(split=False)
        return self._handle_joint

    def __del__(self):
        hs = {id(h): h for h in (getattr(self, "_handle", None), getattr(self, "_handle_joint", None),
                                 *self.__dict__.get("_shard_handles", {}).values())
              if h is not None and h.value}
        for h in hs.values():
            try:
                N.load_library().pgm_rows_plan_destroy(h)
            except Exception:
                pass

    # ------------------------------------------------------------------ run
    def alloc_outputs(self, n_rows, marginals=True, joint=False, map_=False, gap=False):
        import torch

        dev = E.device()
        out = {}
        if marginals:
            out["marg"] = torch.empty((self.n_acc, n_rows), dtype=torch.float64, device=dev)
        if joint:
            out["joint"] = torch.empty((self.P, n_rows), dtype=torch.float64, device=dev)
        if map_ or gap:
            out["map"] = torch.empty(n_rows, dtype=torch.int32, device=dev)
        if gap and self.kind == "fused":
            out["gap"] = torch.empty(n_rows, dtype=torch.float64, device=dev)
        return out

    def run(self, codes, ld, row0, n_rows, out, err=None):
        """Run the plan on rows [row0, row0+n_rows) of the column-major uint8 codes [n_cols, ld].

        out: dict from alloc_outputs (marg [n_acc, n], joint [P, n], map [n] int32, gap [n])."""
        if n_rows <= 0:
            return out
        if self.kind == "fused":
            if "joint" in out and not self.joint_fused_ok:
                self._run_steps(codes, ld, row0, n_rows, {"joint": out["joint"]}, err)
                rest = {k: v for k, v in out.items() if k != "joint"}
                if rest:
                    self._run_fused(codes, ld, row0, n_rows, rest, err)
                return out
            return self._run_fused(codes, ld, row0, n_rows, out, err)
        return self._run_steps(codes, ld, row0, n_rows, out, err)

    def _mode(self, out):
        mode = self.extra_mode
        if "marg" in out:
            mode |= N.ROWS_MARGINALS
        if "joint" in out:
            mode |= N.ROWS_JOINT
        if "map" in out:
            mode |= N.ROWS_MAP
        if "gap" in out:
            mode |= N.ROWS_MAPGAP
        return mode

    def _run_fused(self, codes, ld, row0, n_rows, out, err):
        L = N.lib()
        self._build_fused()
        mode = self._mode(out)
        if (mode & N.ROWS_JOINT) and self.n_comp > 1:
            # the joint over independent components needs the single-component (monolithic) plan
            N.check(L.pgm_rows_plan_run(self._joint_handle(), N.ROWS_JOINT, N.ptr(codes), int(ld), int(row0),
                                        int(n_rows), None, N.ptr(out["joint"]), int(out["joint"].stride(0)), None,
                                        None, N.ptr(err), N.stream_handle()), "rows_plan_run")
            mode &= ~N.ROWS_JOINT
            if not mode:
                return out
        ld_out = n_rows
        if "marg" in out:
            ld_out = int(out["marg"].stride(0))
        elif "joint" in out and (mode & N.ROWS_JOINT):
            ld_out = int(out["joint"].stride(0))
        N.check(L.pgm_rows_plan_run(self._handle, mode, N.ptr(codes), int(ld), int(row0), int(n_rows),
                                    N.ptr(out.get("marg")), N.ptr(out.get("joint")) if mode & N.ROWS_JOINT else None,
                                    int(ld_out), N.ptr(out.get("map")), N.ptr(out.get("gap")), N.ptr(err),
                                    N.stream_handle()), "rows_plan_run")
        return out

    def bind(self, codes, ld, row0, n_rows, out, err=None, stream=None, floor=False):
        """A prepared launch of run() on fixed buffers (pgm_rows_plan_bind): `.run()` re-runs the same
        pass with one argument-free C call.  Fused plans with marginal / MAP outputs only.
        floor=True binds the plan's dispatch floor instead (PGM_ROWS_FLOOR: the same grid, code loads and
        output stores without the CPT arithmetic) — a measurement, its outputs are not results."""
        if self.kind != "fused" or "joint" in out:
            raise ValueError("bind(): fused plans without a joint output only")
        self._build_fused()
        return BoundRows(self, codes, ld, row0, n_rows, out, err, stream, floor=floor)

    def compact(self):
        """This plan reading a compact codes array that holds only the evidence columns it uses, in
        ev_used order (column i = ev_used[i]) — what ingestion uploads when it copies just the columns
        a pattern reads.  Shares the pruning, factors and sources (so is_current() agrees); compiles
        its own kernels.  Cached on the plan."""
        import copy

        c = self.__dict__.get("_compact")
        if c is None:
            with self._lock:
                c = self.__dict__.get("_compact")
                if c is None:
                    c = copy.copy(self)
                    for k in ("_handle", "_handle_joint", "_plan", "_progs", "_compact", "_ev_sel"):
                        c.__dict__.pop(k, None)
                    c._handle = None
                    c._handle_joint = None
                    c._lock = threading.RLock()
                    c.col_of = {v: i for i, v in enumerate(self.ev_used)}
                    self._compact = c
        return c

    def ring(self, slots, n_rows, err=None, stream=None):
        """A resident ring over equally sized row batches (pgm_rows_ring_*): slots = [(codes, ld, row0,
        out), ...]; batch b reads rows [row0, row0 + n_rows) of slot b % len(slots)'s codes and writes
        its outputs (marginal / MAP / gap dicts from alloc_outputs, one per slot).  See RowRing."""
        if self.kind != "fused":
            raise ValueError("ring(): fused plans only")
        self._build_fused()
        return RowRing(self, slots, n_rows, err, stream)

    def _dev_factors(self):
        if not hasattr(self, "_dev_cache"):
            self._dev_cache = [(cpd._d(), vars_) for vars_, cpd in self.factors]
        return self._dev_cache

    def intermediates_per_row(self):
        """(largest, total) intermediate entries per evidence row of the steps path."""
        if not hasattr(self, "_inter"):
            labels, dims = [], dict(self.card)
            dims[E.ROW] = 1
            for vars_, _ in self.factors:
                ls = [v for v in vars_ if v not in self.evidence_vars]
                if any(v in self.evidence_vars for v in vars_):
                    ls = ls + [E.ROW]
                labels.append(ls)
            st = plan_stats(labels, self.variables + [E.ROW], dims)
            self._inter = (max(1, st["max_intermediate"]), max(1, st["sum_intermediate"]))
        return self._inter

    def path_stats(self, n_rows=1):
        """SURVEY.md §8(d) C2 accounting of the steps path for n_rows rows: pairwise steps,
        algorithmic bytes (sum of 8 (|A| + |B| + |C|)), flops (2 |index space|), max intermediate;
        plus how many steps run as dense FP64 MFMA GEMMs."""
        from .contraction import FUSE, _specialising, compiled_path

        fuse = FUSE and _specialising()  # the compiled programs run the fused path (contract_factors)
        labels, dims = [], dict(self.card)
        dims[E.ROW] = n_rows
        for vars_, _ in self.factors:
            ls = [v for v in vars_ if v not in self.evidence_vars]
            if any(v in self.evidence_vars for v in vars_):
                ls = ls + [E.ROW]
            labels.append(ls)
        st = plan_stats(labels, self.variables + [E.ROW], dims, fuse=fuse)
        plan, _, levels = compiled_path(labels, self.variables + [E.ROW], dims, fuse=fuse)
        st["fused"] = fuse
        st["nary_steps"] = sum(1 for p_, _ in plan if p_[0] == "nary")
        st["gemm_steps"] = sum(1 for _, shape in plan if shape is not None and shape != "pack")
        st["packed_steps"] = sum(1 for _, shape in plan if shape == "pack")
        st["levels"] = len(levels)
        return st

    def max_intermediate_per_row(self):
        return self.intermediates_per_row()[0]

    def _steps_chunk(self, n_rows):
        """Rows per compiled steps program: every intermediate is preallocated, so bound both the
        largest one (2^26 entries) and their sum (2^28 entries = 2 GiB)."""
        mx, tot = self.intermediates_per_row()
        return max(1, min(n_rows, (1 << 26) // mx, (1 << 28) // tot))

    def _steps_program(self, n, outs, host_io=False):
        """The steps path for n rows compiled once: evidence gathers from the plan's own codes
        buffer, the greedy contraction (dense steps on FP64 MFMA), normalisation and the requested
        outputs into preallocated buffers, captured as one HIP graph.  host_io: the codes buffer and the
        outputs are host memory the kernels access directly (QueryRunner via query_one).  Returns (program, codes buffer, error flag, outputs, device column
        map, host buffers or None)."""
        progs = self.__dict__.setdefault("_progs", {})
        hit = progs.get((n, outs, host_io))
        if hit is not None:
            return hit
        import torch

        from ..program import Program

        dev = E.device()
        L = N.lib()
        prog = Program()
        ev_set = set(self.evidence_vars)
        cols = list(self.ev_used)
        local = {v: i for i, v in enumerate(cols)}
        perr = torch.zeros(1, dtype=torch.int32, device=dev)
        host = None
        if host_io:
            # the evidence codes and the result live in pinned, mapped, coherent host memory that the
            # kernels read and write directly (pgm_host_alloc): a query is one graph launch + one
            # synchronize, no copy of any size on either side
            host = {"codes": N.HostBuffer((max(1, len(cols)), n), np.uint8)}
            codes_buf = host["codes"].tensor
        else:
            codes_buf = torch.zeros((max(1, len(cols)), n), dtype=torch.uint8, device=dev)
        ops = []
        prog.begin_batch()  # every factor's evidence slice: one launch
        for t, vars_ in self._dev_factors():
            rem = [v for v in vars_ if v not in ev_set]
            dyn = {v: (None, local[v]) for v in vars_ if v in ev_set}
            if dyn:
                g = prog.gather(t, vars_, dyn, rem + [E.ROW], codes_buf, n, 0, n, perr)
                ops.append((g, rem + [E.ROW]))
            else:
                ops.append((t, list(vars_)))
        prog.end_batch()
        outl = self.variables + [E.ROW]
        if not any(E.ROW in ls for _, ls in ops):
            # no evidence touches this pattern: broadcast one result over the rows
            ops.append((E.to_device(np.ones(n)), [E.ROW]))
        R = contract_factors(ops, outl, prog=prog)  # [Q..., ROW] C-order
        # normalisation in two launches whatever the number of query variables: the row masses Z and
        # every variable's unnormalised marginal (all read only R) as one batch, then every division as
        # one batch (before: 1 + 2 V dependent launches of ~4.5 us each).  A single query variable's
        # marginal is R itself (same labels, same layout), not a copy of it.
        prog.begin_batch()
        Z = prog.contract(R, outl, None, None, [E.ROW], reduce="sum", combine="copy")
        ms = []
        if "marg" in outs:
            for v in self.variables:
                ms.append(R if len(self.variables) == 1 else
                          prog.contract(R, outl, None, None, [v, E.ROW], reduce="sum", combine="copy"))
        prog.end_batch()
        bufs = {}

        def out_buf(key, shape):
            if host_io:
                host[key] = N.HostBuffer(tuple(shape), np.float64)
                return host[key].tensor
            return E.empty(list(shape))

        prog.begin_batch()
        if "marg" in outs:
            bufs["marg"] = out_buf("marg", [self.n_acc, n])
            for i, v in enumerate(self.variables):
                a = self.acc_off[i]
                prog.contract(ms[i], [v, E.ROW], Z, [E.ROW], [v, E.ROW], combine="div_raw",
                              out=bufs["marg"][a:a + self.cards[i]])
        if "joint" in outs:
            bufs["joint"] = out_buf("joint", [self.P, n])
            prog.contract(R.reshape(self.P, n), ["q", E.ROW], Z, [E.ROW], ["q", E.ROW], combine="div_raw",
                          out=bufs["joint"])
        if host_io:
            # the single-query program also hands out the joint BEFORE normalisation (the reference's
            # contract result, ExactInference.py:404-406, ahead of normalize at L420): one more job of
            # this last batch, no extra launch; query_one(..., unnorm=True) returns it
            bufs["unnorm"] = out_buf("unnorm", [self.P, n])
            prog.contract(R.reshape(self.P, n), ["q", E.ROW], None, None, ["q", E.ROW], combine="copy",
                          out=bufs["unnorm"])
        prog.end_batch()
        if "map" in outs:
            bufs["map"] = torch.empty(n, dtype=torch.int32, device=dev)
            prog.argmax(R, n, self.P, 1, n, bufs["map"])
        prog.capture()
        cols_dev = torch.tensor([self.col_of[v] for v in cols], dtype=torch.int32, device=dev) if cols else None
        hit = (prog, codes_buf, perr, bufs, cols_dev, host)
        progs[(n, outs, host_io)] = hit
        return hit

    def prepare_steps(self, n, outs, host_io=False):
        """Build (and capture) the steps program for (n, outs, host_io) unless it exists.  The capture
        holds engine.device_lock exclusively, taken BEFORE this plan's own lock: a thread inside a
        public call gives its shared hold up while it waits, and holds no per-plan lock then, so no
        thread holding the device lock shared can be waiting for a lock this one holds."""
        progs = self.__dict__.get("_progs")
        if progs is not None and (n, outs, host_io) in progs:
            return
        with E.device_lock.exclusive():
            with self._lock:
                self._steps_program(n, outs, host_io)

    def prepare_run(self, n_rows, keys):
        """Every captured program run(n_rows rows, outputs `keys`) will replay, built now (see
        prepare_steps): callers that take a lock of their own around run() call this first."""
        keys = set(keys)
        if self.kind == "fused":
            if "joint" not in keys or self.joint_fused_ok:
                return
            keys = {"joint"}
        outs = frozenset(k for k in ("marg", "joint", "map") if k in keys)
        chunk = self._steps_chunk(n_rows)
        for n in {min(chunk, n_rows - c0) for c0 in range(0, n_rows, chunk)}:
            self.prepare_steps(n, outs)

    def query_one(self, codes, key, stream=None, unnorm=False, codes_bytes=None):
        """One evidence row (codes[col_of[v]]: the state number of evidence variable v, already checked
        against the state names on the host) through the steps program whose codes and result live in
        host memory the kernels access directly: fill the codes, one graph launch, one synchronize.
        Returns a new fp64 ndarray (`key` "marg" or "joint"); with unnorm=True the pair (that, the
        unnormalised joint [P] the same program computed before dividing by its mass)."""
        L = N.lib()
        with self._lock:
            q1 = self.__dict__.get("_q1")  # key -> (program, host buffers) of the one-row host-io program
            hit = q1.get(key) if q1 is not None else None
            if hit is None:
                prog, _, _, _, _, host = self._steps_program(1, frozenset([key]), host_io=True)
                self.__dict__.setdefault("_q1", {})[key] = hit = (prog, host)
            prog, host = hit
            if codes_bytes is not None:  # the ev_used codes, in order (one byte per column of the [cols, 1] buffer)
                if len(codes_bytes) != len(self.ev_used):
                    raise ValueError("query_one: one code per evidence column the plan reads")
                if codes_bytes:
                    ctypes.memmove(host["codes"].array.ctypes.data, codes_bytes, len(codes_bytes))
            else:
                sel = self.__dict__.get("_ev_sel")
                if sel is None:  # the caller's column of each evidence variable the plan reads (col_of)
                    idx = [self.col_of[v] for v in self.ev_used]
                    sel = self._ev_sel = ((lambda c, i=idx[0]: (c[i],)) if len(idx) == 1 else
                                          itemgetter(*idx) if idx else None)
                if sel is not None:
                    host["codes"].array[:, 0] = sel(codes)
            if prog._direct or ((dq := DirectQueue.for_queries()) is not None and prog.bind_direct(dq)):
                # the steps as one chain of AQL packets: written and rung in ~2 us, returns when the
                # results are in host memory (a graph launch spends ~17 us on the host first)
                prog.run_direct()
            else:  # the graph on the calling thread's own stream (engine.thread_stream) unless one is given
                stream = stream if stream is not None else E.thread_stream()
                s = N.stream_handle(stream)
                prog.run(stream)
                N.check(L.pgm_stream_sync_spin(s), "stream_sync_spin")  # latency-bound: poll, don't block
            if unnorm:
                return host[key].array.reshape(-1).copy(), host["unnorm"].array.reshape(-1).copy()
            return host[key].array.reshape(-1).copy()

    def _run_steps(self, codes, ld, row0, n_rows, out, err):
        """Batched greedy contraction with an evidence-row axis: rows in chunks, each chunk one
        replay of a compiled program (_steps_program)."""
        outs = frozenset(k for k in ("marg", "joint", "map") if k in out)
        chunk = self._steps_chunk(n_rows)
        for n in {min(chunk, n_rows - c0) for c0 in range(0, n_rows, chunk)}:
            self.prepare_steps(n, outs)  # captures first, before this plan's lock
        with self._lock:  # the compiled programs own their scratch buffers: one caller at a time
            return self._run_steps_locked(codes, ld, row0, n_rows, out, err)

    def _run_steps_locked(self, codes, ld, row0, n_rows, out, err):
        L = N.lib()
        s = N.stream_handle()
        outs = frozenset(k for k in ("marg", "joint", "map") if k in out)
        chunk = self._steps_chunk(n_rows)
        for c0 in range(0, n_rows, chunk):
            n = min(chunk, n_rows - c0)
            prog, cbuf, perr, bufs, cols_dev, _ = self._steps_program(n, outs)
            if cols_dev is not None:
                N.check(L.pgm_codes_select(N.ptr(codes), int(ld), int(row0 + c0), N.ptr(cols_dev), len(self.ev_used),
                                           int(n), N.ptr(cbuf), s), "codes_select")
            N.check(L.pgm_memset(N.ptr(perr), 0, 4, s), "memset")
            prog.run()
            if "marg" in out:
                E.contract(bufs["marg"], ["a", E.ROW], None, None, ["a", E.ROW], combine="copy",
                           out=out["marg"][:, c0:c0 + n])
            if "joint" in out:
                E.contract(bufs["joint"], ["q", E.ROW], None, None, ["q", E.ROW], combine="copy",
                           out=out["joint"][:, c0:c0 + n])
            if "map" in out:
                N.check(L.pgm_memcpy_d2d(N.ptr(out["map"][c0:c0 + n]), N.ptr(bufs["map"]), 4 * n, s), "memcpy")
            if err is not None and int(perr.item()) != 0:
                N.check(L.pgm_memset(N.ptr(err), 1, 4, s), "memset")
        return out

    # ------------------------------------------------------------------ accounting
    def algorithmic_bytes_per_row(self, marginals=True, map_=False, joint=False):
        """HBM bytes per row the plan must move: evidence codes read + outputs written
        (7 B + 136 B marginals or + 3 B MAP codes)."""
        b = len(self.ev_used)
        if marginals:
            b += 8 * self.n_acc
        if joint:
            b += 8 * self.P
        if map_:
            b += len(self.variables)  # one uint8 state code per MAP variable
        return b

    def describe(self):
        return {"kind": self.kind, "components": len(self.components()) if self.kind == "fused" else None,
                "factors": [list(v) for v, _ in self.factors], "hidden": self.hidden,
                "evidence_columns": len(self.ev_used), "query_space": self.P, "hidden_space": self.H,
                "values": int(sum(int(np.prod(c.cardinality)) for _, c in self.factors))}


class QueryRunner:
    """One evidence row through a compiled plan, results back on the host (VariableElimination.query
    on a Bayesian network, ExactInference.py:246-457): the plan's steps program with its codes and
    results in mapped host memory (PatternPlan.query_one — one AQL chain on the query queue, or one graph
    replay), whatever the plan's kind.  r05: fused plans took the fused row kernel here (codes up, the
    pass, results down on the thread's stream: 0.44 ms per query on alarm, against 25 us for the steps
    program; profiles/r05ao/).  A lock makes concurrent queries from several threads on one
    VariableElimination safe (the reference calls map_query from joblib threads on one object,
    DiscreteBayesianNetwork.py:871)."""

    def __init__(self, plan, joint):
        self.plan = plan
        self.joint = bool(joint)
        self.lock = threading.Lock()
        self.key = "joint" if joint else "marg"

    def run_bytes(self, codes):
        """run() with the codes of plan.ev_used already as bytes, in that order (_FastQuery)."""
        if not self.__dict__.get("_prepared"):
            self.plan.prepare_steps(1, frozenset([self.key]), host_io=True)
            self._prepared = True
        with self.lock:
            return self.plan.query_one(None, self.key, codes_bytes=codes)

    def bytes_caller(self):
        """run_bytes once the one-row program is bound to the query queue, as a closure with every lookup
        made once: copy the codes into the mapped host buffer, run the AQL chain, copy the result out
        (r06, _FastQuery's repeat calls).  None while the program is not built or not on the queue."""
        plan = self.plan
        hit = (plan.__dict__.get("_q1") or {}).get(self.key)
        if hit is None or not hit[0]._direct:
            return None
        prog, host = hit
        run = N.lib().pgm_dq_run_chain
        arr, ind, cnt = prog._direct_arr, prog._direct_indep, len(prog._direct)
        dst, n = host["codes"].array.ctypes.data, len(plan.ev_used)
        out = host[self.key].array.reshape(-1)
        memmove, lock, plock = ctypes.memmove, self.lock, plan._lock

        def call(codes):
            if len(codes) != n:
                raise ValueError("query_one: one code per evidence column the plan reads")
            with lock, plock:
                if n:
                    memmove(dst, codes, n)
                if run(arr, ind, cnt):
                    N.check(1, "dq_run_chain")
                return out.copy()

        call.keep = (prog, host)  # the chain's launches and buffers live as long as the closure
        return call

    def run(self, codes, unnorm=False):
        """codes: state numbers of plan.evidence_vars (in that order). Returns a new fp64 ndarray:
        the normalised joint [P] (C-order over plan.variables) or the marginals [n_acc]; with
        unnorm=True also the unnormalised joint [P] of the same run (PatternPlan.query_one)."""
        # the program is built and captured before this runner's lock is taken (engine.DeviceLock)
        if not self.__dict__.get("_prepared"):
            self.plan.prepare_steps(1, frozenset([self.key]), host_io=True)
            self._prepared = True
        with self.lock:
            return self.plan.query_one(codes, self.key, unnorm=unnorm)


class BoundRows:
    """Prepared fused row-plan launch (pgm_rows_plan_bind / pgm_rows_bound_run).  Keeps the plan and
    every buffer alive for as long as the bound handle exists."""

    def __init__(self, plan, codes, ld, row0, n_rows, out, err, stream, floor=False):
        import ctypes

        L = N.lib()
        self._keep = (plan, codes, out, err)
        mode = plan._mode(out) | (N.ROWS_FLOOR if floor else 0)
        ld_out = int(out["marg"].stride(0)) if "marg" in out else int(n_rows)
        h = ctypes.c_void_p()
        N.check(L.pgm_rows_plan_bind(plan._handle, mode, N.ptr(codes), int(ld), int(row0), int(n_rows),
                                     N.ptr(out.get("marg")), None, ld_out, N.ptr(out.get("map")),
                                     N.ptr(out.get("gap")), N.ptr(err), N.stream_handle(stream), ctypes.byref(h)),
                "rows_plan_bind")
        self._h = h
        self._run = L.pgm_rows_bound_run
        self.out = out

    def run(self):
        st = self._run(self._h)
        if st != 0:
            N.check(st, "rows_bound_run")
        return self.out

    def kernel(self):
        """(kernel name, blocks, workgroup size) this bound launch runs (pgm_rows_bound_kernel);
        the name is "" for an AOT kernel."""
        import ctypes

        name = ctypes.create_string_buffer(64)
        nb, wg = ctypes.c_uint32(), ctypes.c_uint32()
        N.check(N.lib().pgm_rows_bound_kernel(self._h, name, 64, ctypes.byref(nb), ctypes.byref(wg)),
                "rows_bound_kernel")
        return name.value.decode(), nb.value, wg.value

    def direct(self, queue=None):
        """The same launch dispatched on a DirectQueue (pgm_dq_bind_rows): one AQL packet per
        run(), no HIP runtime on the launch path.  Needs the plan-specialised kernel."""
        return DirectRows(self, queue or DirectQueue.default())

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                N.load_library().pgm_rows_bound_destroy(h)
            except Exception:
                pass


class RowRing:
    """One resident launch of the plan-specialised row kernel consuming a stream of row batches
    (pgm_rows_ring_*; DESIGN.md "Resident ring").  start(n) launches it for n batches, post(k) publishes
    batches [0, k) (a batch's inputs must be complete on the device and its slot's previous batch
    finished), finish() waits for the launch.  Outputs equal run()'s on the same rows bit for bit."""

    def __init__(self, plan, slots, n_rows, err, stream):
        import ctypes

        L = N.lib()
        slots = list(slots)
        if not slots:
            raise ValueError("RowRing: no slots")
        outs = [s[3] for s in slots]
        mode = plan._mode(outs[0])
        if any(plan._mode(o) != mode for o in outs):
            raise ValueError("RowRing: every slot needs the same outputs")
        n = len(slots)
        P = ctypes.c_void_p
        codes = (P * n)(*[s[0].data_ptr() for s in slots])
        lds = (ctypes.c_int64 * n)(*[int(s[1]) for s in slots])
        row0 = (ctypes.c_int64 * n)(*[int(s[2]) for s in slots])

        def ptrs(key):
            if key not in outs[0]:
                return None
            return (P * n)(*[o[key].data_ptr() for o in outs])

        ld_out = int(outs[0]["marg"].stride(0)) if "marg" in outs[0] else int(n_rows)
        if "marg" in outs[0] and any(int(o["marg"].stride(0)) != ld_out for o in outs):
            raise ValueError("RowRing: every slot's marginals need the same leading dimension")
        h = ctypes.c_void_p()
        N.check(L.pgm_rows_ring_create(plan._handle, mode, n, codes, lds, row0, int(n_rows), ptrs("marg"), ld_out,
                                       ptrs("map"), ptrs("gap"), N.ptr(err), N.stream_handle(stream),
                                       ctypes.byref(h)), "rows_ring_create")
        self._keep = (plan, slots, err)
        self._h = h
        self._post = L.pgm_rows_ring_post
        self._n, self._posted = -1, 0  # no launch yet: a post is refused by the library
        self._start = L.pgm_rows_ring_start
        ptr, base = ctypes.c_void_p(), ctypes.c_uint32()
        N.check(L.pgm_rows_ring_counter(h, ctypes.byref(ptr), ctypes.byref(base)), "rows_ring_counter")
        # the pinned host counter as a one-element uint32 array: a post is one aligned store
        self._counter = np.ctypeslib.as_array((ctypes.c_uint32 * 1).from_address(ptr.value))
        self._base = base.value
        self.outs = outs
        self.n_rows = int(n_rows)
        self.n_slots = n

    def start(self, n_batches, timeout_s=5.0, wait_ready=False):
        """Launch for n_batches batches; wait_ready=True returns only once every workgroup of the
        resident grid is running (pgm_rows_ring_start_ready)."""
        base = int(self._counter[0])  # the launch's base: batches posted over the ring's lifetime
        if wait_ready:
            N.check(N.lib().pgm_rows_ring_start_ready(self._h, int(n_batches), float(timeout_s), float(timeout_s)),
                    "rows_ring_start_ready")
        else:
            N.check(self._start(self._h, int(n_batches), float(timeout_s)), "rows_ring_start")
        self._base = base
        self._n = int(n_batches)
        self._posted = 0

    def post(self, n_posted):
        """Publish batches [0, n_posted) of the running launch: one store into the pinned counter
        (pgm_rows_ring_counter; the same as pgm_rows_ring_post without a library call).  Batch b runs on
        slot b % n_slots: a caller refilling a slot for batch b + n_slots must know batch b is done
        (finish() of the launch that ran it); within one launch, repeats of a slot read the same inputs."""
        if not self._posted <= n_posted <= self._n:
            st = self._post(self._h, int(n_posted))  # the library reports the misuse
            N.check(st, "rows_ring_post")
        self._posted = n_posted
        self._counter[0] = self._base + n_posted

    def finish(self):
        N.check(N.lib().pgm_rows_ring_finish(self._h), "rows_ring_finish")

    def cancel(self):
        N.check(N.lib().pgm_rows_ring_cancel(self._h), "rows_ring_cancel")

    def kernel(self):
        """(kernel name, resident blocks, workgroup size)."""
        import ctypes

        name = ctypes.create_string_buffer(64)
        nb, wg = ctypes.c_uint32(), ctypes.c_uint32()
        N.check(N.lib().pgm_rows_ring_kernel(self._h, name, 64, ctypes.byref(nb), ctypes.byref(wg)),
                "rows_ring_kernel")
        return name.value.decode(), nb.value, wg.value

    def run(self, n_batches, timeout_s=5.0, replay=False):
        """start + post every batch + finish (one resident launch over n_batches batches).  Batches are
        posted at once, so batch b and batch b + n_slots may run concurrently on the same slot:
        n_batches > n_slots is refused unless replay=True, the caller's statement that every slot's
        inputs stay unchanged for the whole launch (the repeats then write identical outputs — a
        bandwidth measurement, bench.py's single-launch roofline)."""
        if int(n_batches) > self.n_slots and not replay:
            raise ValueError(f"RowRing.run: {n_batches} batches over {self.n_slots} slots would run a slot's "
                             f"repeats concurrently; refill slots between launches or pass replay=True")
        self.start(n_batches, timeout_s)
        try:
            for b in range(1, int(n_batches) + 1):
                self.post(b)
        except BaseException:
            self.cancel()
            raise
        self.finish()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                N.load_library().pgm_rows_ring_destroy(h)
            except Exception:
                pass


class DirectQueue:
    """A user-mode HSA queue on the current HIP device (pgm_dq_create, pgmpy_amd/csrc/pgmdq.cpp).
    Dispatches on it run in order; sync() before HIP work reads their outputs."""

    _default = {}

    def __init__(self, device=None):
        import ctypes

        import torch

        self.device = torch.cuda.current_device() if device is None else int(device)
        h = ctypes.c_void_p()
        N.check(N.lib().pgm_dq_create(self.device, ctypes.byref(h)), "dq_create")
        self._h = h

    @classmethod
    def default(cls):
        import torch

        d = torch.cuda.current_device()
        q = cls._default.get(d)
        if q is None:
            q = cls._default[d] = cls(d)
        return q

    _queries = {}

    @classmethod
    def for_queries(cls):
        """The current device's queue for compiled single queries (Program.bind_direct / run_direct; its
        own queue), or None when PGM_QUERY_DIRECT=0 or the queue cannot be made (the queries then replay
        their HIP graphs).

        r06: the queue keeps its dispatch timestamps ON.  r05 switched them off here
        (pgm_dq_profiling(q, 0)) and the chain then crashed rocprofv3, so queries bypassed the queue
        under the profiler.  A kernel-tracing tool intercepts every queue, puts its own completion
        signal on each dispatch and reads that dispatch's start/end with
        hsa_amd_profiling_get_dispatch_time, which needs profiling enabled on the queue the packets run
        on; turning it off on an intercepted queue takes away the timestamps the tool relies on.  Only a
        chain's last packet carries a signal of ours, so the timestamps cost the chain nothing."""
        import torch

        if os.environ.get("PGM_QUERY_DIRECT", "1") == "0":
            return None
        d = torch.cuda.current_device()
        q = cls._queries.get(d, False)
        if q is False:
            try:
                q = cls(d)
            except RuntimeError:
                q = None
            cls._queries[d] = q
        return q

    @property
    def handle(self):
        return self._h

    def sync(self):
        N.check(N.lib().pgm_dq_sync(self._h), "dq_sync")

    def release(self):
        """Append the system-scope release barrier without waiting (pgm_dq_release; wait() then
        covers it): several queues release in parallel."""
        N.check(N.lib().pgm_dq_release(self._h), "dq_release")

    def wait(self):
        """Every dispatch issued so far has completed (no release: sync() before HIP reads)."""
        N.check(N.lib().pgm_dq_wait(self._h), "dq_wait")

    def timer_start(self):
        N.check(N.lib().pgm_dq_timer_start(self._h), "dq_timer_start")

    def timer_stop_ms(self):
        import ctypes

        ms = ctypes.c_float()
        N.check(N.lib().pgm_dq_timer_stop_ms(self._h, ctypes.byref(ms)), "dq_timer_stop")
        return float(ms.value)

    def timer_stop_ticks(self):
        """(start, end, ticks per second) of the timed span (pgm_dq_timer_stop_ticks)."""
        import ctypes

        a, b, f = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        N.check(N.lib().pgm_dq_timer_stop_ticks(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(f)),
                "dq_timer_stop")
        return a.value, b.value, f.value

    def dispatch_times(self, cap=4096):
        """[(start, end)] ticks of each dispatch of the last timed span, in issue order
        (pgm_dq_timer_dispatch_times; the frequency is timer_stop_ticks()'s third value)."""
        import ctypes

        a = (ctypes.c_uint64 * cap)()
        b = (ctypes.c_uint64 * cap)()
        n = ctypes.c_int32()
        N.check(N.lib().pgm_dq_timer_dispatch_times(self._h, a, b, cap, ctypes.byref(n)), "dq_timer_dispatch_times")
        return [(a[i], b[i]) for i in range(n.value)]

    def dispatch_stats(self):
        """(sum of the last timed span's per-dispatch durations in ticks, dispatches summed)."""
        import ctypes

        t, n = ctypes.c_uint64(), ctypes.c_uint64()
        N.check(N.lib().pgm_dq_timer_dispatch_stats(self._h, ctypes.byref(t), ctypes.byref(n)),
                "dq_timer_dispatch_stats")
        return t.value, n.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                N.load_library().pgm_dq_destroy(h)
            except Exception:
                pass


class DirectGroup:
    """Bound launches on one DirectQueue whose outputs are pairwise distinct (independent row
    batches), dispatched together by pgm_dq_launch_group: the first packet waits for all earlier
    work, the others may overlap it, so one batch's workgroups start while the previous drains."""

    def __init__(self, members):
        import ctypes

        members = list(members)
        if not members:
            raise ValueError("DirectGroup: no launches")
        q = members[0].queue
        if any(m.queue is not q for m in members):
            raise ValueError("DirectGroup: launches bound to different queues")
        spans = []  # byte range each member's outputs cover (views of one buffer may overlap)
        for i, m in enumerate(members):
            for t in m.out.values():
                if t.numel() == 0:
                    continue
                last = sum((int(d) - 1) * int(st) for d, st in zip(t.shape, t.stride()) if int(st) > 0)
                spans.append((t.data_ptr(), t.data_ptr() + (last + 1) * t.element_size(), i))
        for k, (a0, a1, i) in enumerate(spans):
            for b0, b1, j in spans[k + 1:]:
                if i != j and a0 < b1 and b0 < a1:
                    raise ValueError("DirectGroup: launches write overlapping output bytes")
        self._keep = members
        self.queue = q
        self._arr = (ctypes.c_void_p * len(members))(*[m._h.value for m in members])
        self._n = len(members)
        self._launch = N.lib().pgm_dq_launch_group

    def run(self):
        st = self._launch(self._arr, self._n)
        if st != 0:
            N.check(st, "dq_launch_group")

    def sync(self):
        self.queue.sync()


class DirectRows:
    """A bound row-plan launch re-bound to a DirectQueue (pgm_dq_bind_rows / pgm_dq_launch)."""

    def __init__(self, bound, queue):
        import ctypes

        self._keep = (bound, queue)
        self.queue = queue
        self.out = bound.out
        h = ctypes.c_void_p()
        N.check(N.lib().pgm_dq_bind_rows(queue._h, bound._h, ctypes.byref(h)), "dq_bind_rows")
        self._h = h
        self._launch = N.lib().pgm_dq_launch

    def run(self):
        st = self._launch(self._h)
        if st != 0:
            N.check(st, "dq_launch")
        return self.out

    def run_release(self):
        """The launch with a system-scope release on its own completion (pgm_dq_launch_release): the last
        launch before the outputs are read; wait with queue.wait()."""
        N.check(N.lib().pgm_dq_launch_release(self._h), "dq_launch_release")
        return self.out

    def sync(self):
        self.queue.sync()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                N.load_library().pgm_dq_bound_destroy(h)
            except Exception:
                pass
