"""Fixed launch sequences with preallocated buffers, replayed or captured as one HIP graph.

A Program records device launches (pgm_contract / pgm_product_n / pgm_indicator
/ pgm_gather) with their descriptors, operand pointers and workspaces resolved
at build time; run() replays them (one ctypes call each) and capture() records
them into a HIP graph (pgm_graph_capture_*) so a whole compiled schedule — a
batched BP calibration, a fixed-shape contraction plan — is one launch.
"""
import ctypes
import os

from . import _native as N
from . import engine as E
from . import hazard as H


# index-space size (outputs x reduction) up to which a step joins a batch
BATCH_MAX_WORK = 1 << 22
# a step the planner would split (few outputs, long reduction) joins only this small
BATCH_SPLIT_WORK = 1 << 16
# the same for a plain Program's batches (the levels of a contraction path, C1 / C2): a split step costs two
# launches (partials + final) at ~4.5 us each, more than the unsplit job takes inside the level's batch — C2
# 0.218 -> 0.204 ms/query (profiles/r03w/)
PLAIN_SPLIT_WORK = 1 << 22
# plain Program: a lone contraction up to this index space becomes a batch of one (specialised kernel)
LONE_BATCH_WORK = 1 << 16
# outputs up to which an n-ary product joins a level batch (flat mode, 8-B accesses); larger ones keep
# their own row-mode launch (16-B two-rows-per-lane).  2 M best of 64 K / 512 K / 2 M / 4 M / 8 M
# (profiles/r01i_c4_variants.txt); 256 K / 64 K within noise (r03ak)
PRODN_BATCH_MAX = 1 << 21
# levelled programs: n-ary products / separator marginals at least this large (entries) become
# specialised steps merged per level instead of level-batch jobs (the bind declines shapes it cannot
# take or that are below the engine's own threshold)
# C4 1,000 rows: 0.97 -> 1.03M (r03ag, 2^14); r06at: 2^12 with the generator's own threshold, +0.5-0.7 %
PM_PREFER_MIN = int(os.environ.get("PGM_PM_PREFER_MIN", 1 << 12))
PM_MERGE_BODIES = int(os.environ.get("PGM_PM_MERGE_BODIES", 64))  # pgm_pm_merge takes up to 128; 128 measured neutral on C4 (r06n)
# plain programs: consecutive dependency levels of at most this many 256-thread blocks each, all of their
# jobs contractions, run in ONE single-workgroup launch (pgm_batch_set_mode ONE_WORKGROUP, k_batch_wg_c:
# descriptors staged in LDS, a level's blocks four at a time in a 1,024-thread workgroup, a workgroup
# barrier between levels) instead of one launch each — the tail of a contraction path (C1 / C2: the last
# levels down to the query marginal, then its normalisation).  C2 0.173-0.174 against 0.179 ms, C1 0.067
# against 0.069-0.071 (profiles/r04o/; 8 or more blocks per level: C1 slower).  0 = one launch per level.
# (r03's persistent grid-barrier form of several levels and its one-block-at-a-time generic chain were
# measured slower and removed in r05.)  r05: replayed as graphs the chain won on C1 (0.062 -> 0.056 ms/query)
# and lost on C2 (0.123 -> 0.128 ms), so _tune_chains timed both forms per program; dispatched as one AQL
# chain (the single-query default since) the chain wins on both — C2 0.111-0.112 vs 0.122-0.124 ms, C1 0.049
# vs 0.060 (profiles/r05ae/) — so programs keep the chain; CHAIN_TUNE = True times both as graphs.  Levels of up
# to 8 blocks chained (r05aq, after every single query took the chain): C1 0.0255 -> 0.0245 ms, C2 unchanged.
WG_CHAIN_BLOCKS = 8
CHAIN_TUNE = False
# plain programs: every level batch of contractions (and the single-workgroup chain) runs as ONE
# plan-specialised kernel (pgm_batch_specialise) instead of the descriptor-driven k_batch_c /
# k_batch_wg_c (r05).  A/B knob PGM_BATCH_RTC=0
BATCH_SPECIALISE = os.environ.get("PGM_BATCH_RTC", "1") != "0"
# A/B knob: a level batch of more jobs than this as that many jobs per kernel, the parts independent packets
# (0: one kernel per level unless over the kernel-argument budget)
PART_JOBS = int(os.environ.get("PGM_PART_JOBS", 0))


def _key(t):
    """Hazard identity of a device tensor: its storage (views of one buffer conflict)."""
    return t.untyped_storage().data_ptr()


class _Rec:
    """One recorded launch of a levelled Program: plain launch, optional batch job, buffers it
    reads / writes (storage keys)."""

    __slots__ = ("fn", "note", "job", "reads", "writes", "level", "pm", "nbytes", "foot", "step")

    def __init__(self, fn, note, job, reads, writes, pm=None, nbytes=0, foot=None, step=0):
        self.fn, self.note, self.job = fn, note, job
        self.reads, self.writes = reads, writes
        self.level = 0
        self.pm = pm  # bound specialised product+marginal step (mergeable with its level's others)
        self.nbytes = nbytes  # algorithmic bytes: every distinct tensor read or written once
        self.foot = foot  # byte ranges the launch touches, from its descriptor (hazard.py)
        self.step = step  # plain Program: the launch this record runs in (a batch's jobs share one)


class _PMStep:
    """A launch of one plan-specialised kernel (pgm_pm_bound_run: a fused product step, a merged level or
    a specialised contraction batch), or of several independent ones (a level batch over the kernel-argument
    budget, in parts); `bounds` are their handles, which a direct AQL chain re-binds (Program.bind_direct)."""

    __slots__ = ("bounds", "batch")

    def __init__(self, *bounds):
        self.bounds = bounds
        self.batch = None  # the level batch it runs, when it runs one (profiling: Program.time_step_jobs)

    def __call__(self, s):
        L = N.lib()
        for b in self.bounds:
            N.check(L.pgm_pm_bound_run(b, s), "pm_bound_run")


class _Batch:
    """Independent small jobs collected between Program.begin_batch() and end_batch()."""

    def __init__(self):
        self.jobs = []  # (kind, batch args, plain-launch args)


class Program:
    """levels=True: launches are recorded with the buffers they read and write and, before the first
    run / capture, grouped into dependency levels (a step's level is one past every earlier step it
    must follow: read-after-write, write-after-read, write-after-write).  Each level is its big steps'
    own launches plus ONE pgm_batch launch of all its small jobs (contractions, gathers, n-ary
    products): a batched BP sweep becomes ~2 launches per tree level instead of ~4 per clique."""

    def __init__(self, levels=False):
        self._levels = levels
        self._recs = []
        self._lowered = False
        self._steps = []
        self._keep = []
        self._graph = None
        self._stream = None
        self._batch = None
        self._handles = []
        self._pm_bound = []  # specialised product+marginal kernels (pgm_product_n_marginal_bind)
        self._pm_prepared = 0  # plain Program: _pm_bound[:n] compiled by _ready
        self._chain_alts = []  # plain Program: (single-workgroup chain step, [(fn, note) per level]) not yet tuned
        self.step_levels = []  # levelled Program: the dependency level of each lowered step
        self.step_bytes = []  # levelled Program: algorithmic bytes of each lowered step (profiling aid)
        self._pm_launch = None  # the specialised steps actually launched (compiled by _ready)
        self.notes = []  # one short description per step (profiling aid: tools/program_steps.py)
        self.merged_parts = {}  # step index -> full notes of the specialised steps merged into it
        self.merged_handles = {}  # step index -> the merged steps' own bound handles (profiling aid)
        self._plain_recs = []  # plain Program: one record per launch / batch job (check_hazards only)
        self._unit = 0  # plain Program: launch counter behind _Rec.step
        self._plain_lowered = -1  # plain Program: len(_steps) right after the last lowering
        self._direct = None  # bind_direct: the steps' direct AQL launches, () when not eligible
        self.direct_note = None

    # ------------------------------------------------------------------ batching
    def begin_batch(self):
        """Small contractions / gathers recorded until end_batch() become ONE launch
        (pgm_batch_*); the caller guarantees they are independent of each other."""
        if self._batch is not None:
            raise RuntimeError("batch already open")
        self._batch = _Batch()
        self._unit += 1  # every job of the batch runs in the same launch

    def end_batch(self):
        """Close the batch.  It becomes a step when the program is lowered (first run / capture):
        consecutive batches (the levels of a contraction path, each reading the ones before) run as
        ONE levelled batch launch; a lone batch is one launch, a batch of one the job's own launch."""
        b, self._batch = self._batch, None
        if b is None or not b.jobs:
            return
        self._steps.append(b)
        self.notes.append(f"batch of {len(b.jobs)}")

    def raw_step(self, fn, note):
        """Append a launch `fn(stream)` as is (plain Program; e.g. a stream-ordered host copy that the
        captured graph then holds as a memcpy node)."""
        if self._levels:
            raise RuntimeError("raw_step: plain Program only")
        self._unit += 1
        self._steps.append(fn)
        self.notes.append(note)

    @staticmethod
    def _add_batch_jobs(h, jobs):
        L = N.lib()
        for kind, args, _ in jobs:
            if kind == "contract":
                N.check(L.pgm_batch_add_contract(h, *args), "batch_add_contract")
            elif kind == "contract_n":
                N.check(L.pgm_batch_add_contract_n(h, *args), "batch_add_contract_n")
            else:
                N.check(L.pgm_batch_add_gather(h, *args), "batch_add_gather")

    def _batch_blocks(self, b):
        """256-thread blocks the jobs of batch b occupy inside a single-workgroup levelled batch (planned
        on a scratch handle in that mode)."""
        L = N.lib()
        h = ctypes.c_void_p()
        N.check(L.pgm_batch_create(ctypes.byref(h)), "batch_create")
        try:
            N.check(L.pgm_batch_set_mode(h, N.BATCH_ONE_WORKGROUP), "batch_set_mode")
            self._add_batch_jobs(h, b.jobs)
            n = ctypes.c_int64()
            N.check(L.pgm_batch_blocks(h, ctypes.byref(n)), "batch_blocks")
            return int(n.value)
        finally:
            L.pgm_batch_destroy(h)

    def _specialise(self, h):
        """The finalized batch h as one plan-specialised kernel (pgm_batch_specialise: literal shapes,
        strides and block ranges, no descriptor reads), or None when it does not take the batch."""
        if not BATCH_SPECIALISE:
            return None
        b = ctypes.c_void_p()
        N.check(N.lib().pgm_batch_specialise(h, ctypes.byref(b)), "batch_specialise")
        if not b.value:
            return None
        self._pm_bound.append(b)
        return b

    def _specialise_parts(self, jobs, max_jobs=0):
        """A level batch whose kernel arguments exceed one specialised kernel's budget (512 pointers: a
        contraction takes 3, a gather 4; C2's 205-gather level) as consecutive parts that each fit, every
        part specialised; None when there is nothing to split or a part is not taken."""
        if not BATCH_SPECIALISE or len(jobs) < 2:
            return None
        chunks, cur, n = [], [], 0
        for j in jobs:
            w = 4 if j[0] == "gather" else (j[1][0]._obj.n_ops + 1) if j[0] == "contract_n" else 3
            if cur and (n + w > 512 or (max_jobs and len(cur) >= max_jobs)):
                chunks.append(cur)
                cur, n = [], 0
            cur.append(j)
            n += w
        chunks.append(cur)
        if len(chunks) < 2:
            return None
        L = N.lib()
        out = []
        for c in chunks:
            h = self._new_batch()
            self._add_batch_jobs(h, c)
            N.check(L.pgm_batch_finalize(h), "batch_finalize")
            sb = self._specialise(h)
            if sb is None:
                return None
            out.append(sb)
        return out

    def _batch_step(self, b):
        L = N.lib()
        if PART_JOBS and len(b.jobs) > PART_JOBS:
            parts = self._specialise_parts(b.jobs, PART_JOBS)
            if parts:
                st = _PMStep(*parts)
                st.batch = b
                return st, f"specialised batch of {len(b.jobs)} in {len(parts)} parts"
        h = self._new_batch()
        self._add_batch_jobs(h, b.jobs)
        N.check(L.pgm_batch_finalize(h), "batch_finalize")
        sb = self._specialise(h)
        if sb is not None:
            st = _PMStep(sb)
            st.batch = b
            return st, f"specialised batch of {len(b.jobs)}"
        parts = self._specialise_parts(b.jobs)
        if parts:
            st = _PMStep(*parts)
            st.batch = b
            return st, f"specialised batch of {len(b.jobs)} in {len(parts)} parts"
        if any(kind == "contract_n" for kind, _, _ in b.jobs):
            raise RuntimeError("a batch with n-ary contraction jobs was not specialised (hipRTC unavailable or "
                               "PGM_NO_JIT set); contraction.FUSE plans them only when it is")
        if len(b.jobs) == 1:  # a job the generator does not take: its own planner's launch
            kind, _, args = b.jobs[0]
            if kind == "contract":
                return (lambda s, a=args: N.check(L.pgm_contract(*a, s), "contract")), "contract (batch of one)"
            return (lambda s, a=args: N.check(L.pgm_gather(*a, s), "gather")), "gather (batch of one)"
        return (lambda s, hh=h: N.check(L.pgm_batch_run(hh, s), "batch_run")), f"batch of {len(b.jobs)}"

    def _chain_batch(self, group):
        """A single-workgroup levelled batch of `group`'s levels (contractions only), or None when its
        staged tables exceed the kernel's LDS budget (pgm_batch_finalize: PGM_EINVAL)."""
        L = N.lib()
        h = ctypes.c_void_p()
        N.check(L.pgm_batch_create(ctypes.byref(h)), "batch_create")
        try:
            N.check(L.pgm_batch_set_mode(h, N.BATCH_ONE_WORKGROUP), "batch_set_mode")
            for m, b in enumerate(group):
                if m:
                    N.check(L.pgm_batch_add_level(h), "batch_add_level")
                self._add_batch_jobs(h, b.jobs)
            if L.pgm_batch_finalize(h) != 0:
                L.pgm_batch_destroy(h)
                return None
        except Exception:
            L.pgm_batch_destroy(h)
            raise
        self._handles.append(h)
        return h

    def _lower_batches(self):
        """Plain Program: closed batches -> launches (see end_batch)."""
        if not any(isinstance(s, _Batch) for s in self._steps):
            return
        L = N.lib()
        steps, notes = [], []
        i, n = 0, len(self._steps)
        while i < n:
            if not isinstance(self._steps[i], _Batch):
                steps.append(self._steps[i])
                notes.append(self.notes[i])
                i += 1
                continue
            j = i
            while j < n and isinstance(self._steps[j], _Batch):
                j += 1
            group = self._steps[i:j]
            if WG_CHAIN_BLOCKS > 0 and len(group) >= 2:
                # runs of consecutive tiny levels of contractions (each at most WG_CHAIN_BLOCKS blocks) ->
                # one single-workgroup launch; the other levels keep one launch each
                blocks = [self._batch_blocks(b) if all(kind in ("contract", "contract_n") for kind, _, _ in b.jobs)
                          else None for b in group]
                k = 0
                while k < len(group):
                    e = k
                    while e < len(group) and blocks[e] is not None and blocks[e] <= WG_CHAIN_BLOCKS:
                        e += 1
                    if e - k >= 2:
                        h = self._chain_batch(group[k:e])
                        if h is not None:
                            sb = self._specialise(h)
                            if sb is not None:
                                fn = _PMStep(sb)
                            elif any(kind == "contract_n" for b in group[k:e] for kind, _, _ in b.jobs):
                                raise RuntimeError("a single-workgroup chain with n-ary contraction jobs was not "
                                                   "specialised")
                            else:
                                fn = lambda s, hh=h: N.check(L.pgm_batch_run(hh, s), "batch_run")
                            steps.append(fn)
                            notes.append(f"{e - k} levels in one workgroup ({sum(blocks[k:e])} blocks, "
                                         f"{sum(len(b.jobs) for b in group[k:e])} jobs)")
                            # the same levels one launch each: _tune_chains keeps whichever form is faster
                            # (built only when it will tune: each alternative is a specialised kernel that
                            # _ready would otherwise compile and keep unused)
                            if CHAIN_TUNE:
                                self._chain_alts.append((fn, [self._batch_step(b) for b in group[k:e]]))
                            k = e
                            continue
                        e = k + 1  # tables over the LDS budget: one launch per level
                    fn, note = self._batch_step(group[k])
                    steps.append(fn)
                    notes.append(note)
                    k += 1
            else:
                for b in group:
                    fn, note = self._batch_step(b)
                    steps.append(fn)
                    notes.append(note)
            i = j
        self._steps, self.notes = steps, notes

    # ------------------------------------------------------------------ levelled recording
    @staticmethod
    def _rec(fn, note, reads, writes, job=None, pm=None, foot=None, step=0):
        rk = [k for k in (_key(t) for t in reads if t is not None) if k]
        wk = [k for k in (_key(t) for t in writes if t is not None) if k]
        seen, nb = set(), 0
        for t in list(reads) + list(writes):
            if t is not None and hasattr(t, "numel") and id(t) not in seen:
                seen.add(id(t))
                nb += t.numel() * t.element_size()
        return _Rec(fn, note, job, rk, wk, pm, nb, foot, step)

    def _emit(self, fn, note, reads, writes, job=None, pm=None, foot=None):
        """Append one launch (plain `fn(stream)`), or record it for levelling.  reads / writes: the
        buffers the launch declares (its hazards); foot: the byte ranges its descriptor touches
        (hazard.py), checked against the declarations by check_hazards()."""
        if self._levels:
            if self._lowered:
                raise RuntimeError("levelled Program: no recording after the first run / capture")
            self._recs.append(self._rec(fn, note, reads, writes, job, pm, foot))
        else:
            self._unit += 1
            self._plain_recs.append(self._rec(fn, note, reads, writes, foot=foot, step=self._unit))
            self._steps.append(fn)
            self.notes.append(note)

    def _batch_job(self, note, reads, writes, foot):
        """Plain Program: record a job of the open batch for check_hazards()."""
        self._plain_recs.append(self._rec(None, note, reads, writes, foot=foot, step=self._unit))

    def check_hazards(self):
        """Recompute every recorded launch's byte ranges from its descriptor and check them against
        the declared reads / writes and the launch order the program runs (hazard.check): [] when
        every overlap is ordered.  Host only (no launch)."""
        self._lower()
        recs = self._recs if self._levels else self._plain_recs
        units = [(r.note, r.foot or [], r.reads, r.writes, None) for r in recs]
        tensors = [t for t in self._keep if hasattr(t, "untyped_storage")]
        if self._levels:
            return H.check(units, tensors, lambda a, b: recs[b].level > recs[a].level)
        return H.check(units, tensors, lambda a, b: recs[a].step != recs[b].step)

    def _ready(self):
        """Lower, then compile every specialised kernel the steps launch (in parallel, before any
        run or capture)."""
        self._lower()
        if self._pm_launch is None or not self._levels:  # plain Program: every bound step not yet prepared
            self._pm_launch = self._pm_bound[self._pm_prepared:]
            self._pm_prepared = len(self._pm_bound)
        if self._pm_launch:
            arr = (ctypes.c_void_p * len(self._pm_launch))(*[h.value for h in self._pm_launch])
            N.check(N.lib().pgm_pm_prepare(arr, len(self._pm_launch)), "pm_prepare")
            self._pm_launch = []
        if self._chain_alts:
            if CHAIN_TUNE:
                self._tune_chains()
            else:
                self._chain_alts = []

    def _tune_chains(self, reps=20):
        """A run of tiny dependent levels goes faster as one single-workgroup launch on some programs (C1:
        0.062 -> 0.056 ms/query) and slower on others (C2: 0.123 -> 0.128 ms): capture the whole program
        both ways as HIP graphs (how compiled queries replay it), time `reps` replays of each, alternately,
        best of two, and keep the faster.  The steps recompute the same outputs from the same inputs, so
        the extra replays change nothing."""
        import torch

        alts, self._chain_alts = self._chain_alts, []
        chained = (list(self._steps), list(self.notes))
        swap = {id(fn): lv for fn, lv in alts}
        flat = ([], [])
        for fn, note in zip(*chained):
            for f, n in swap.get(id(fn), [(fn, note)]):
                flat[0].append(f)
                flat[1].append(n)
        L = N.lib()
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        graphs = []
        with E.device_lock.exclusive():
            torch.cuda.current_stream().synchronize()
            st = torch.cuda.Stream()
            s = N.stream_handle(st)
            N.check(L.pgm_event_create(ctypes.byref(a)))
            N.check(L.pgm_event_create(ctypes.byref(b)))
            try:
                for steps in (chained[0], flat[0]):
                    g = ctypes.c_void_p()
                    N.check(L.pgm_graph_capture_begin(s), "graph_capture_begin")
                    try:
                        for step in steps:
                            step(s)
                    finally:
                        N.check(L.pgm_graph_capture_end(s, ctypes.byref(g)), "graph_capture_end")
                    graphs.append(g)

                def timed(g):
                    N.check(L.pgm_graph_launch(g, s), "graph_launch")
                    N.check(L.pgm_event_record(a, s))
                    for _ in range(reps):
                        N.check(L.pgm_graph_launch(g, s), "graph_launch")
                    N.check(L.pgm_event_record(b, s))
                    ms = ctypes.c_float()
                    N.check(L.pgm_event_elapsed_ms(a, b, ctypes.byref(ms)))
                    return ms.value

                t_chain = t_flat = float("inf")
                for _ in range(2):
                    t_chain = min(t_chain, timed(graphs[0]))
                    t_flat = min(t_flat, timed(graphs[1]))
                st.synchronize()
            finally:
                for g in graphs:
                    L.pgm_graph_destroy(g)
                L.pgm_event_destroy(a)
                L.pgm_event_destroy(b)
        self.chain_tuning = {"chained_us": t_chain * 1e3 / reps, "per_level_us": t_flat * 1e3 / reps}
        if t_flat < t_chain:
            self._steps, self.notes = flat
            self._plain_lowered = len(self._steps)

    def _lower(self):
        """Levelled Program -> steps: per level, its unbatched launches then one batch launch."""
        if not self._levels:
            if len(self._steps) != self._plain_lowered:  # steps recorded since the last lowering
                self._lower_batches()
                self._plain_lowered = len(self._steps)
            return
        if self._lowered:
            return
        self._lowered = True
        self._pm_launch = []
        last_w, last_r = {}, {}
        n_lv = 0
        for r in self._recs:
            lv = 0
            for k in r.reads:
                lv = max(lv, last_w.get(k, -1) + 1)
            for k in r.writes:
                lv = max(lv, last_w.get(k, -1) + 1, last_r.get(k, -1) + 1)
            r.level = lv
            n_lv = max(n_lv, lv + 1)
            for k in r.reads:
                last_r[k] = max(last_r.get(k, -1), lv)
            for k in r.writes:
                last_w[k] = max(last_w.get(k, -1), lv)
        by_level = [[] for _ in range(n_lv)]
        for r in self._recs:
            by_level[r.level].append(r)
        for lv, recs in enumerate(by_level):
            self._emit_level(lv, recs)

    @staticmethod
    def _add_jobs(h, recs):
        L = N.lib()
        for r in recs:
            kind, args = r.job
            if kind == "contract":
                N.check(L.pgm_batch_add_contract(h, *args), "batch_add_contract")
            elif kind == "gather":
                N.check(L.pgm_batch_add_gather(h, *args), "batch_add_gather")
            elif kind == "indicator":
                N.check(L.pgm_batch_add_indicator(h, *args), "batch_add_indicator")
            else:
                N.check(L.pgm_batch_add_product_n(h, *args), "batch_add_product_n")

    def _new_batch(self):
        h = ctypes.c_void_p()
        N.check(N.lib().pgm_batch_create(ctypes.byref(h)), "batch_create")
        self._handles.append(h)
        return h

    def _emit_level(self, lv, recs):
        """One dependency level: its unbatched launches, then one batch launch of its small jobs."""
        small = [r for r in recs if r.job is not None]
        n0 = len(self._steps)
        # (r05: launching the large steps alone, or ordering the merged bodies by size, measured slower:
        # -6 to -18 % at 4,000 rows, profiles/r05g/)
        merged = self._merge_pm([r for r in recs if r.job is None and r.pm is not None])
        for r in recs:
            if r in merged:
                continue
            if r.job is None or len(small) == 1:
                self._steps.append(r.fn)
                self.notes.append(r.note)
                self.step_bytes.append(r.nbytes)
                if r.pm is not None:
                    self._pm_launch.append(r.pm)
        if len(small) < 2:
            self.step_levels.extend([lv] * (len(self._steps) - n0))
            return
        L = N.lib()
        h = self._new_batch()
        self._add_jobs(h, small)
        N.check(L.pgm_batch_finalize(h), "batch_finalize")
        self._steps.append(lambda s, hh=h: N.check(L.pgm_batch_run(hh, s), "batch_run"))
        self.notes.append(f"level batch of {len(small)}: " + "; ".join(r.note[:60] for r in small[:4]))
        self.step_bytes.append(sum(r.nbytes for r in small))
        self.step_levels.extend([lv] * (len(self._steps) - n0))

    def _merge_pm(self, recs):
        """A level's specialised product+marginal steps as one launch per 64 (pgm_pm_merge); returns
        the records merged (their launches are emitted here; one launch per step: -21 % / -35 % at
        4,000 / 1,000 rows of C4, profiles/r04v/)."""
        if len(recs) < 2:
            return set()
        L = N.lib()
        done = set()
        parts, cur, n_ptr = [], [], 0
        for r in recs:  # <= PM_MERGE_BODIES bodies and <= 512 kernel-argument pointers (operands + C + M) per launch
            k = len(r.reads) + 2
            if cur and (len(cur) == PM_MERGE_BODIES or n_ptr + k > 512):
                parts.append(cur)
                cur, n_ptr = [], 0
            cur.append(r)
            n_ptr += k
        parts.append(cur)
        for part in parts:
            if len(part) < 2:
                continue
            arr = (ctypes.c_void_p * len(part))(*[r.pm.value for r in part])
            m = ctypes.c_void_p()
            N.check(L.pgm_pm_merge(arr, len(part), ctypes.byref(m)), "pm_merge")
            if not m.value:
                continue
            self._pm_bound.append(m)
            self._pm_launch.append(m)
            self.merged_parts[len(self._steps)] = [r.note for r in part]
            self.merged_handles[len(self._steps)] = [r.pm for r in part]
            self._steps.append(_PMStep(m))
            self.notes.append(f"merged {len(part)} specialised steps: " + "; ".join(r.note[:60] for r in part[:3]))
            self.step_bytes.append(sum(r.nbytes for r in part))
            done.update(part)
        return done

    @property
    def n_levels(self):
        self._lower()
        return 1 + max((r.level for r in self._recs), default=-1)

    # ------------------------------------------------------------------ recording
    def contract(self, A, la, B, lb, out_labels, reduce=None, combine="mul", out=None):
        d, out, ws, wsb = E.prepare_contract(A, la, B, lb, out_labels, reduce, combine, out)
        self._keep.extend([d, A, B, out, ws])
        L = N.lib()
        note = f"contract {combine}/{reduce} {list(la)}{tuple(A.shape)} x {lb} -> {list(out_labels)}"
        if self._levels:
            w = _work(d)
            args = (ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(out), N.ptr(ws), wsb)
            job = None
            if w <= (BATCH_MAX_WORK if wsb == 0 else BATCH_SPLIT_WORK):
                job = ("contract", (ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(out)))
            fn, pm = (lambda s, a=args: N.check(L.pgm_contract(*a, s), "contract")), None
            foot = H.contract_foot(d, N.ptr(A), N.ptr(B), N.ptr(out), N.ptr(ws), wsb)
            if (job is None or A.numel() >= PM_PREFER_MIN) and B is None and combine == "copy" and \
                    reduce in ("sum", "max"):
                bm = self._bind_marginal(A, la, out_labels, out, reduce)
                if bm is not None:
                    pm, foot = bm
                    fn, job = _PMStep(pm), None
            self._emit(fn, note, [A, B], [out, ws], job, pm=pm, foot=foot)
            return out
        w = _work(d)
        if self._batch is None and wsb == 0 and w <= LONE_BATCH_WORK:
            # a small lone contraction (a single query's final transposing copy) as a batch of one: lowered
            # to a plan-specialised kernel like the batched levels, so the program can run as one AQL chain
            self.begin_batch()
            try:
                return self.contract(A, la, B, lb, out_labels, reduce, combine, out)
            finally:
                self.end_batch()
        if self._batch is not None and w <= (BATCH_MAX_WORK if wsb == 0 else PLAIN_SPLIT_WORK):
            self._batch.jobs.append(("contract", (ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(out)),
                                     (ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(out), N.ptr(ws), wsb)))
            self._batch_job(note, [A, B], [out], H.contract_foot(d, N.ptr(A), N.ptr(B), N.ptr(out)))
            return out
        args = (ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(out), N.ptr(ws), wsb)
        self._emit(lambda s, a=args: N.check(L.pgm_contract(*a, s), "contract"), note, [A, B], [out, ws],
                   foot=H.contract_foot(d, N.ptr(A), N.ptr(B), N.ptr(out), N.ptr(ws), wsb))
        return out

    def contract_n(self, operands, out_labels, reduce="sum", out=None):
        """C[out_labels] = REDUCE over the other labels of prod_i X_i (operands: (tensor, labels)) as ONE
        job of the open batch (plain Program; pgm_batch_add_contract_n, specialised kernel only): a fused
        group of a contraction path's pairwise steps (contraction.fuse_path)."""
        if self._levels or self._batch is None:
            raise RuntimeError("contract_n: a job of an open batch of a plain Program")
        d, ptrs, out = E.prepare_contract_n(operands, out_labels, reduce, out)
        self._keep.extend([d, ptrs, out] + [t for t, _ in operands])
        self._batch.jobs.append(("contract_n", (ctypes.byref(d), ptrs, N.ptr(out)), None))
        note = f"contract_n {reduce} {len(operands)} ops -> {list(out_labels)}"
        self._batch_job(note, [t for t, _ in operands], [out], H.contract_n_foot(d, ptrs, N.ptr(out)))
        return out

    def _bind_marginal(self, A, la, out_labels, out, reduce):
        """(bound, footprint): out = reduce of A onto out_labels as a specialised marginal-only step (one
        operand), or None when the fused kernel does not take the shape (rows not innermost, too few
        blocks)."""
        la, out_labels = list(la), list(out_labels)
        if not out_labels or out_labels[-1] != la[-1] or any(l not in la for l in out_labels):
            return None
        d, ptrs, _, ms, _, ok = E.prepare_product_n_marginal([(A, la)], la, out_labels, out=A, store=False,
                                                             M=out)
        if not ok:
            return None
        L = N.lib()
        bound = ctypes.c_void_p()
        N.check(L.pgm_product_n_marginal_bind(ctypes.byref(d), ptrs, None, ms, E._REDUCE[reduce], N.ptr(out),
                                              ctypes.byref(bound)), "product_n_marginal_bind")
        if not bound.value:
            return None
        self._keep.extend([d, ptrs, ms])
        self._pm_bound.append(bound)
        return bound, H.product_n_foot(d, ptrs, None, store=False, marg=[(ms, N.ptr(out))])

    def product_n(self, operands, out_labels, out=None, kinds=None):
        ops = list(operands)
        kinds = list(kinds) if kinds is not None else [N.PRODN_MUL] * len(ops)
        L = N.lib()
        if len(ops) > N.PRODN_MAX_OPS and all(k == N.PRODN_MUL for k in kinds):
            # more operands than one kernel takes: a balanced tree of products (independent groups of
            # up to PRODN_MAX_OPS, then their partial products) instead of a sequential fold, so a
            # levelled program runs the groups in one level — pathfinder's root folds 46 one-variable
            # messages: 2 dependency levels instead of 7
            m = N.PRODN_MAX_OPS
            n_groups = -(-len(ops) // m)
            size = -(-len(ops) // n_groups)
            partials = [(self.product_n(ops[i:i + size], out_labels), list(out_labels))
                        for i in range(0, len(ops), size)]
            return self.product_n(partials, out_labels, out)
        while len(ops) > N.PRODN_MAX_OPS:  # fold the surplus (plain MUL operands) into the output first
            cut = N.PRODN_MAX_OPS if kinds[N.PRODN_MAX_OPS - 1] != N.PRODN_RATIO else N.PRODN_MAX_OPS - 1
            out = self.product_n(ops[:cut], out_labels, out, kinds[:cut])
            ops = [(out, list(out_labels))] + ops[cut:]
            kinds = [N.PRODN_MUL] + kinds[cut:]
        d, ptrs, out = E.prepare_product_n(ops, out_labels, out, kinds)
        self._keep.extend([d, ptrs, out] + [t for t, _ in ops])
        args = (ctypes.byref(d), ptrs, N.ptr(out))
        job = ("product_n", args) if out.numel() <= PRODN_BATCH_MAX else None
        fn, pm = (lambda s, a=args: N.check(L.pgm_product_n(*a, s), "product_n")), None
        if (job is None or out.numel() >= PM_PREFER_MIN) and self._levels and len(ops) <= N.PM_MAX_OPS:
            # a specialised step, merged with its level's
            bound = ctypes.c_void_p()
            N.check(L.pgm_product_n_bind(*args, ctypes.byref(bound)), "product_n_bind")
            if bound.value:
                self._pm_bound.append(bound)
                fn, pm, job = _PMStep(bound), bound, None
        self._emit(fn, f"product_n {[(list(ls), tuple(t.shape), tuple(t.stride())) for t, ls in ops]} "
                       f"-> {list(out_labels)}{tuple(out.shape)}", [t for t, _ in ops], [out], job, pm=pm,
                   foot=H.product_n_foot(d, ptrs, N.ptr(out)))
        return out

    def product_n_marginal(self, operands, out_labels, marg_labels, out=None, kinds=None, reduce="sum",
                           store=True):
        """Recorded C = product_n(...) with M = reduce(C) onto marg_labels in the same pass
        (pgm_product_n_marginal) when the fused kernel applies, else product_n + contract.
        store=False asks for M alone: the fused kernel then writes nothing to C (the fallback
        still materialises C).  Returns (C, M, stored)."""
        ops = list(operands)
        if len(ops) <= N.PM_MAX_OPS:
            d, ptrs, out2, ms, M, ok = E.prepare_product_n_marginal(ops, out_labels, marg_labels, out, kinds, store)
            if ok:
                L = N.lib()
                self._keep.extend([d, ptrs, out2, ms, M] + [t for t, _ in ops])
                args = (ctypes.byref(d), ptrs, N.ptr(out2) if store else None, ms, E._REDUCE[reduce], N.ptr(M))
                bound = ctypes.c_void_p()
                N.check(L.pgm_product_n_marginal_bind(*args, ctypes.byref(bound)), "product_n_marginal_bind")
                pm = None
                if bound.value:  # the plan compiled into a specialised kernel
                    self._pm_bound.append(bound)
                    pm = bound
                    fn = _PMStep(bound)
                else:
                    fn = lambda s, a=args: N.check(L.pgm_product_n_marginal(*a, s), "product_n_marginal")
                self._emit(fn,
                           f"product_n_marginal{'' if store else ' (marginal only)'} "
                           f"{[(list(ls), tuple(t.shape)) for t, ls in ops]} "
                           f"-> {list(out_labels)}{tuple(out2.shape)} + {list(marg_labels)}{tuple(M.shape)}",
                           [t for t, _ in ops], [out2, M] if store else [M], pm=pm,
                           foot=H.product_n_foot(d, ptrs, N.ptr(out2), store, [(ms, N.ptr(M))]))
                return out2, M, store
        C = self.product_n(ops, out_labels, out, kinds)
        M = self.contract(C, list(out_labels), None, None, list(marg_labels), reduce=reduce, combine="copy")
        return C, M, True

    def product_n_marginals(self, operands, out_labels, marg1, marg2, out=None, kinds=None, reduce="sum"):
        """(M1, M2): two marginals of the product of operands onto marg1 / marg2 in ONE specialised
        pass that stores nothing else (pgm_product_n_marginals_bind), or None when the pass does not
        take the shapes.  `out` (not written) only describes the product's index space."""
        ops = list(operands)
        if len(ops) > N.PM_MAX_OPS or not self._levels:
            return None
        L = N.lib()
        d, ptrs, C = E.prepare_product_n(ops, out_labels, out, kinds)
        shape = {l: int(C.shape[i]) for i, l in enumerate(out_labels)}
        Ms, strides = [], []
        for marg in (marg1, marg2):
            M = E.empty([shape[l] for l in marg])
            Ms.append(M)
            strides.append((ctypes.c_int64 * len(out_labels))(*[int(M.stride(list(marg).index(l))) if l in marg else 0
                                                                 for l in out_labels]))
        bound = ctypes.c_void_p()
        N.check(L.pgm_product_n_marginals_bind(ctypes.byref(d), ptrs, strides[0], N.ptr(Ms[0]), strides[1],
                                               N.ptr(Ms[1]), E._REDUCE[reduce], ctypes.byref(bound)),
                "product_n_marginals_bind")
        if not bound.value:
            return None
        self._keep.extend([d, ptrs, C] + strides + Ms + [t for t, _ in ops])
        self._pm_bound.append(bound)
        self._emit(_PMStep(bound),
                   f"product_n_marginals {[(list(ls), tuple(t.shape)) for t, ls in ops]} -> {list(marg1)} + "
                   f"{list(marg2)}", [t for t, _ in ops], Ms, pm=bound,
                   foot=H.product_n_foot(d, ptrs, None, store=False,
                                         marg=[(strides[0], N.ptr(Ms[0])), (strides[1], N.ptr(Ms[1]))]))
        return Ms[0], Ms[1]

    def indicator(self, codes_col, card, n_rows, err=None):
        out = E.empty([card, n_rows])
        L = N.lib()
        args = (N.ptr(codes_col), int(n_rows), int(card), N.ptr(out), int(out.stride(0)), int(out.stride(1)),
                N.ptr(err))
        self._keep.extend([codes_col, out, err])
        # err is an atomic OR flag: not a hazard; a levelled program batches all findings into one launch
        self._emit(lambda s, a=args: N.check(L.pgm_indicator(*a, s), "indicator"), f"indicator card {card}",
                   [codes_col], [out], ("indicator", args),
                   foot=H.indicator_foot(N.ptr(codes_col), n_rows, card, N.ptr(out), int(out.stride(0)),
                                         int(out.stride(1)), N.ptr(err)))
        return out

    def gather(self, A, la, evidence, out_labels, codes, ld, row0, n_rows, err=None):
        d, Aptr, out = E.prepare_gather(A, la, evidence, out_labels, codes, ld, row0, n_rows)
        L = N.lib()
        args = (ctypes.byref(d), Aptr, N.ptr(codes), N.ptr(out), N.ptr(err))
        self._keep.extend([d, A, codes, out, err])
        note = f"gather {list(la)} -> {list(out_labels)}"
        foot = H.gather_foot(d, Aptr, N.ptr(codes), N.ptr(out), N.ptr(err))
        if self._levels:
            self._emit(lambda s, a=args: N.check(L.pgm_gather(*a, s), "gather"), note,
                       [A, codes], [out], ("gather", args) if out.numel() <= BATCH_MAX_WORK else None, foot=foot)
            return out
        if self._batch is not None and out.numel() <= BATCH_MAX_WORK:
            self._batch.jobs.append(("gather", args, args))
            self._batch_job(note, [A, codes], [out], foot)
            return out
        self._emit(lambda s, a=args: N.check(L.pgm_gather(*a, s), "gather"), note, [A, codes], [out], foot=foot)
        return out

    def pair_gemm(self, A, la, B, lb, keep, shape):
        """Recorded dense step (engine.prepare_gemm): C over `keep`, offset table kept alive."""
        d, table, C = E.prepare_gemm(A, la, B, lb, keep, shape)
        L = N.lib()
        args = (ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(C))
        self._keep.extend([d, table, A, B, C])
        groups = dict(zip(("b", "m", "n", "k"), shape))

        def unit_group(T, ls):  # which group holds the operand's stride-1 variable (layout note)
            for i, l in enumerate(ls):
                if T.stride(i) == 1 and T.shape[i] > 1:
                    return next((g for g, gl in groups.items() if l in gl), "?") + f"({T.shape[i]})"
            return "-"

        self._emit(lambda s, a=args: N.check(L.pgm_gemm(*a, s), "gemm"),
                   f"gemm b{d.batch} m{d.m} n{d.n} k{d.k} unit A:{unit_group(A, la)} B:{unit_group(B, lb)} "
                   f"lane_order {d.lane_order} strides(ab,bb,cb,am,cm,ak,bk,bn,cn)={list(d.stride)}", [A, B, table], [C],
                   foot=H.view_foot(A, H.READ) + H.view_foot(B, H.READ) + H.view_foot(table, H.READ) +
                   H.view_foot(C, H.WRITE))
        return C

    def argmax(self, X, n_rows, row_len, s_row, s_elem, out32):
        L = N.lib()
        args = (N.ptr(X), int(n_rows), int(row_len), int(s_row), int(s_elem), None, N.ptr(out32))
        self._keep.extend([X, out32])
        self._emit(lambda s, a=args: N.check(L.pgm_argmax(*a, s), "argmax"), "argmax", [X], [out32],
                   foot=H.argmax_foot(N.ptr(X), n_rows, row_len, s_row, s_elem, N.ptr(out32)))

    def time_steps(self, reps=3):
        """[(us, note)] per recorded step, each replayed alone (profiling aid; not graph-replayed)."""
        import ctypes as C

        self._ready()
        L = N.lib()
        s = N.stream_handle()
        a, b = C.c_void_p(), C.c_void_p()
        N.check(L.pgm_event_create(C.byref(a)))
        N.check(L.pgm_event_create(C.byref(b)))
        out = []
        for step, note in zip(self._steps, self.notes):
            step(s)
            N.check(L.pgm_event_record(a, s))
            for _ in range(reps):
                step(s)
            N.check(L.pgm_event_record(b, s))
            ms = C.c_float()
            N.check(L.pgm_event_elapsed_ms(a, b, C.byref(ms)))
            out.append((ms.value * 1e3 / reps, note))
        L.pgm_event_destroy(a)
        L.pgm_event_destroy(b)
        return out

    def time_step_jobs(self, i, reps=20):
        """[(us, kind, descriptor summary)] for each job of step i (a specialised level batch), each job
        specialised and replayed alone (profiling aid: which job of a level sets its time)."""
        import ctypes as C

        self._ready()
        st = self._steps[i]
        b = getattr(st, "batch", None)
        if b is None:
            return []
        L = N.lib()
        s = N.stream_handle()
        ev0, ev1 = C.c_void_p(), C.c_void_p()
        N.check(L.pgm_event_create(C.byref(ev0)))
        N.check(L.pgm_event_create(C.byref(ev1)))
        out = []
        for job in b.jobs:
            h = self._new_batch()
            self._add_batch_jobs(h, [job])
            N.check(L.pgm_batch_finalize(h), "batch_finalize")
            sb = self._specialise(h)
            if sb is None:
                continue
            N.check(L.pgm_pm_bound_run(sb, s))
            N.check(L.pgm_event_record(ev0, s))
            for _ in range(reps):
                N.check(L.pgm_pm_bound_run(sb, s))
            N.check(L.pgm_event_record(ev1, s))
            ms = C.c_float()
            N.check(L.pgm_event_elapsed_ms(ev0, ev1, C.byref(ms)))
            d = job[1][0]
            d = getattr(d, "_obj", d)
            if job[0] == "contract_n":
                desc = {"n_ops": int(d.n_ops), "keep": [int(d.keep_card[q]) for q in range(d.n_keep)],
                        "red": [int(d.red_card[q]) for q in range(d.n_red)]}
            elif job[0] == "contract":
                desc = {"keep": [int(d.keep_card[q]) for q in range(d.n_keep)],
                        "red": [int(d.red_card[q]) for q in range(d.n_red)]}
            else:
                desc = {}
            out.append((ms.value * 1e3 / reps, job[0], desc))
        L.pgm_event_destroy(ev0)
        L.pgm_event_destroy(ev1)
        return out

    # ------------------------------------------------------------------ execution
    def run(self, stream=None):
        g = self._graph
        if g is None:  # a captured program was lowered and prepared before its capture
            self._ready()
        s = N.stream_handle(stream)
        if g is not None:
            N.check(N.lib().pgm_graph_launch(g, s), "graph_launch")
        else:
            for step in self._steps:
                step(s)

    @E.exclusive
    def capture(self):
        """Record the steps into one HIP graph (captured on a private stream, holding engine.device_lock
        exclusively: no other thread launches while the stream captures)."""
        import torch

        if self._graph is not None:
            return
        self._ready()
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

    # ------------------------------------------------------------------ direct AQL chain (r05)
    def bind_direct(self, dq):
        """Re-bind every step to the user-mode queue dq (plan.DirectQueue; pgm_dq_bind_pm) so run_direct()
        dispatches the program as one chain of AQL packets: no graph launch on the host (C2: 17.5 us of the
        0.123 ms query before the GPU starts).  Only a plain program whose steps are all plan-specialised
        launches qualifies (at most 128); returns whether this one does.  Bound once per program; the
        reason a program does not qualify is kept in `direct_note`."""
        if self._direct is not None:
            return bool(self._direct)
        self._ready()
        self._direct = ()
        steps = self._steps
        if self._levels or not steps or len(steps) > 128:
            self.direct_note = f"{len(steps)} steps (levelled or over 128)"
            return False
        other = [n for f, n in zip(steps, self.notes) if not isinstance(f, _PMStep)]
        if other:
            self.direct_note = "not specialised: " + "; ".join(other[:3])
            return False
        L = N.lib()
        hs, indep = [], []
        for f in steps:
            for j, b in enumerate(f.bounds):
                d = ctypes.c_void_p()
                if len(hs) >= 128 or L.pgm_dq_bind_pm(dq.handle, b, ctypes.byref(d)) != 0:
                    self.direct_note = "dq_bind_pm: " + (N.last_error() if len(hs) < 128 else "over 128 launches")
                    for h in hs:
                        L.pgm_dq_bound_destroy(h)
                    return False
                hs.append(d)
                indep.append(1 if j else 0)  # a step's parts after its first: independent of each other
        self._direct = hs
        self._direct_q = dq  # the queue outlives the launches bound to it
        self._direct_arr = (ctypes.c_void_p * len(hs))(*[h.value for h in hs])
        self._direct_indep = (ctypes.c_uint8 * len(hs))(*indep)
        self.direct_note = f"{len(hs)} launches as one AQL chain"
        return True

    def run_direct(self):
        """One replay as a chain of AQL packets on the bound queue; returns when the last step has
        completed and its outputs are visible to the host (pgm_dq_run_chain)."""
        N.check(N.lib().pgm_dq_run_chain(self._direct_arr, self._direct_indep, len(self._direct)), "dq_run_chain")

    def __len__(self):
        self._lower()
        return len(self._steps)

    def __del__(self):
        g = getattr(self, "_graph", None)
        try:
            L = N.load_library()
            for h in getattr(self, "_direct", None) or ():
                L.pgm_dq_bound_destroy(h)
            if g is not None and g.value:
                L.pgm_graph_destroy(g)
            for h in getattr(self, "_handles", []):
                L.pgm_batch_destroy(h)
            for h in getattr(self, "_pm_bound", []):
                L.pgm_pm_bound_destroy(h)
        except Exception:
            pass


def _work(d):
    """Index-space size of a contraction descriptor (outputs x reduction)."""
    w = 1
    for i in range(d.n_keep):
        w *= int(d.keep_card[i])
    for i in range(d.n_red):
        w *= int(d.red_card[i])
    return w
