#!/usr/bin/env python3
"""Benchmark: evidence-batched marginal queries/sec on munin (BASELINE.json metric).

Workload: the munin predict_probability template —
missing = random.Random(0).sample(sorted(nodes), 3), evidence = the other 1,038
variables — on synthetic forward-sampled evidence rows (seed 42 + rank),
ROWS per GPU per step (default 100,000 = C3).  One step = one pass of the hot
path over the batch: the compiled fused row plan (pgm_rows_plan_run: evidence
gather -> sum-product -> normalize -> per-variable marginals) reading the
column-major uint8 evidence resident in HBM and writing the [17, rows] fp64
marginals to HBM.

    python bench.py [--gpus N --steps K --warmup W --rows R]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, rows sharded: weak scaling)

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel
(pgm_rows_jit, the plan-specialised kernel, for the C3 template; achieved = algorithmic bytes per launch / HIP-event launch time) and a
CPU baseline (the numpy oracle's per-row predict_probability, single core,
bounded sample) timed on this host.
Other workloads for DESIGN.md numbers: --workload c2 (single munin query,
greedy device contraction) and c4 (pathfinder batched BP calibration).
"""
import argparse
import gc
import ctypes
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
MALL_BYTES = 256 << 20  # MI355X Infinity Cache (memory-side last-level cache)
METRIC = "evidence-batched marginal queries/sec on munin; achieved HBM GB/s vs peak"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


_BACKEND = "nccl"


def dist_setup(n_gpus, backend="auto"):
    """One rank per GPU (torch.distributed.run sets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*).

    backend "nccl" is RCCL on ROCm.  "auto" picks it when every rank has its own GPU, else "gloo"
    (several ranks sharing one GPU: a plumbing rehearsal on the one-GPU box, never a scaling
    number)."""
    global _BACKEND
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={world}: launch N ranks (torchrun) or let "
                         f"bench.py start them itself (WORLD_SIZE unset)")
    if world > 1:
        import torch.distributed as dist

        n_dev = max(1, torch.cuda.device_count())
        dev = local % n_dev
        torch.cuda.set_device(dev)
        if backend == "auto":
            backend = "nccl" if n_dev >= world else "gloo"
        _BACKEND = backend
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        return dist, rank, world
    if torch.cuda.is_available():
        torch.cuda.set_device(0)
    return None, 0, 1


def launch_ranks(n):
    """--gpus N without WORLD_SIZE: start N ranks with torch.distributed.run as a child process.

    This parent never touches the GPU (no HIP call before or after): it only waits for the
    launcher and exits with its status."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log("bench.py: starting", n, "ranks:", " ".join(cmd))
    # rank 0's JSON line is the only stdout line; library chatter (gloo's connection messages go to
    # stdout) is forwarded to stderr
    p = subprocess.Popen(cmd, env=dict(os.environ), stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        if line.lstrip().startswith("{"):
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    return p.wait()


def barrier(dist):
    import torch

    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
        torch.cuda.synchronize()


def max_over_ranks(dist, x):
    if dist is None:
        return x
    import torch

    t = torch.tensor([x], dtype=torch.float64, device="cuda" if _BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class HipTimer:
    """HIP events on the stream the kernels are launched on (pgm_event_*)."""

    def __init__(self):
        from pgmpy_amd import _native as N

        self.N = N
        self.L = N.lib()
        self.a, self.b = ctypes.c_void_p(), ctypes.c_void_p()
        N.check(self.L.pgm_event_create(ctypes.byref(self.a)))
        N.check(self.L.pgm_event_create(ctypes.byref(self.b)))

    def start(self):
        self.N.check(self.L.pgm_event_record(self.a, self.N.stream_handle()))

    def stop_ms(self):
        self.mark_end()
        return self.elapsed_ms()

    def mark_end(self):
        self.N.check(self.L.pgm_event_record(self.b, self.N.stream_handle()))

    def elapsed_ms(self):
        """start -> end event (both complete: call after the stream has been synchronized)."""
        ms = ctypes.c_float()
        self.N.check(self.L.pgm_event_elapsed_ms(self.a, self.b, ctypes.byref(ms)))
        return float(ms.value)


class Launcher:
    """The timed launch of a bound fused row plan.  "direct" (default): one AQL dispatch packet per
    step on a user-mode HSA queue (pgm_dq_launch; kernel time = the queue's dispatch timestamps
    from the first to the last timed dispatch).  "hip": hipModuleLaunchKernel per step
    (pgm_rows_bound_run; kernel time = HIP events on the launch stream).

    Several bounds (distinct row batches, distinct outputs): step i runs batch i % len(bounds);
    with group > 1 (direct only) consecutive steps are dispatched `group` at a time as one
    pgm_dq_launch_group (first packet waits for all earlier work, the others may overlap it)."""

    def __init__(self, bound, kind, group=1, queues=1, qs=None):
        bounds = list(bound) if isinstance(bound, (list, tuple)) else [bound]
        self.kind = kind
        self.group = max(1, int(group))
        queues = max(1, int(queues))
        if (self.group > 1 or queues > 1) and kind != "direct":
            raise ValueError("grouped / multi-queue dispatch needs --launch direct")
        if self.group > 1 and queues > 1:
            raise ValueError("--group and --queues are separate experiments")
        if max(self.group, queues) > len(bounds):
            raise ValueError(f"group / queues of {max(self.group, queues)} need as many distinct batches "
                             f"({len(bounds)} bound)")
        if kind == "direct":
            from pgmpy_amd.inference.plan import DirectQueue

            # batch i on queue i % queues (queue 0: the process's default queue); reuse `qs` when given:
            # every extra user-mode queue costs a hardware queue slot, and past the slots the GPU
            # scheduler time-slices the queues (8 queues: 2x slower than 4, profiles/r02bd_*)
            if qs is not None:
                self.qs = list(qs)[:queues]
            else:
                self.qs = [DirectQueue.default()] + [DirectQueue() for _ in range(queues - 1)]
            self.rs = [b.direct(self.qs[i % queues]) for i, b in enumerate(bounds)]
            self.q = self.qs[0]
        else:
            self.rs = bounds
            self.timer = HipTimer()
        self.r = self.rs[0]
        self._groups = {}
        self._next = 0

    def run(self):
        """One step: the next batch."""
        self.rs[self._next].run()
        self._next = (self._next + 1) % len(self.rs)

    def steps(self, k):
        """k steps, `group` launches per dispatch call when grouped."""
        if self.group == 1:
            for _ in range(k):
                self.run()
            return
        from pgmpy_amd.inference.plan import DirectGroup

        n = len(self.rs)
        while k > 0:
            g = min(self.group, k)
            key = (self._next, g)
            grp = self._groups.get(key)
            if grp is None:
                grp = self._groups[key] = DirectGroup([self.rs[(self._next + j) % n] for j in range(g)])
            grp.run()
            self._next = (self._next + g) % n
            k -= g

    def sync(self):
        import torch

        if self.kind == "direct":
            for q in self.qs:
                q.sync()
        torch.cuda.synchronize()

    def steps_released(self, k):
        """k steps (group 1) whose last launch on each queue releases at system scope on its own
        completion (pgm_dq_launch_release), so the window needs no separate release barrier packet."""
        nq = len(self.qs) if self.kind == "direct" else 0
        if self.group != 1 or nq == 0 or k < nq:
            self.steps(k)
            self._released = False
            return
        last = set()
        n = len(self.rs)
        for j in range(k - nq, k):
            last.add(j)
        for j in range(k):
            r = self.rs[self._next]
            if j in last:
                r.run_release()
            else:
                r.run()
            self._next = (self._next + 1) % n
        # every queue got exactly one released launch when its launches are round robin over the queues
        self._released = len({id(self.rs[(self._next - 1 - t) % n].queue) for t in range(nq)}) == nq

    def release_and_wait(self):
        """End of a timed region with the outputs released at system scope: when the window's last
        launch per queue carried the release (steps_released) just wait; else direct queues append
        their release barriers together, then wait; HIP: wait() (end event + device synchronize)."""
        if self.kind == "direct" and not getattr(self, "_released", False):
            for q in self.qs:
                q.release()
        self._released = False
        self.wait()

    def wait(self):
        """End of a timed region: every launch issued so far has completed (direct queues: their
        completion signals; HIP: the device)."""
        import torch

        if self.kind == "direct":
            for q in self.qs:
                q.wait()
        else:  # the end event goes on the stream right after the last launch
            self._hip_ms = self.timer.stop_ms()
        torch.cuda.synchronize()

    def timer_start(self):
        if self.kind == "direct":
            for q in self.qs:
                q.timer_start()
        else:
            self.timer.start()

    def timer_stop_ms(self):
        if self.kind != "direct":
            ms, self._hip_ms = getattr(self, "_hip_ms", None), None
            return ms if ms is not None else self.timer.stop_ms()
        spans = [q.timer_stop_ticks() for q in self.qs]  # one HSA system clock for every queue
        stats = [q.dispatch_stats() for q in self.qs]
        # the raw per-dispatch timestamps behind the span (tools/c3_span_check.py recomputes the line's
        # kernel_ms and frac from them): [queue, start tick, end tick] in issue order per queue
        self.dispatch_times = {"freq": spans[0][2],
                               "dispatches": [[qi, int(a), int(b)] for qi, q in enumerate(self.qs)
                                              for a, b in q.dispatch_times()]}
        n = sum(c for _, c in stats)
        # each timed dispatch's own duration, averaged: the per-launch figure rocprofv3's kernel trace
        # reports (with several queues it includes the time the dispatch shares the GPU with others)
        self.dispatch_avg_ms = (sum(t for t, _ in stats) * 1e3 / spans[0][2] / n) if n else None
        spans = [(a, b, f) for a, b, f in spans if b > a]
        if not spans:
            return 0.0
        return (max(b for _, b, _ in spans) - min(a for a, _, _ in spans)) * 1e3 / spans[0][2]


def dispatch_floor_ms(plan, d_codes, rows, args, launcher_cls):
    """(floor, kernel): average GPU span per launch of the plan's dispatch floor
    (PatternPlan.bind(floor=True): same grid, loads and stores, no CPT arithmetic) and of the measured
    kernel itself, each over args.steps launches on ONE queue into one output buffer, outside the timed
    region — so the two are compared like for like.  (None, None) when the specialised kernel is not
    in use."""
    if plan.kernel_name() != "pgm_rows_jit":
        return None, None
    res = []
    for floor in (True, False):
        out = plan.alloc_outputs(rows, marginals=True)
        fl = launcher_cls(plan.bind(d_codes, rows, 0, rows, out, floor=floor), args.launch)
        fl.steps(max(args.warmup, 1))
        fl.sync()
        fl.timer_start()
        fl.steps(args.steps)
        ms = fl.timer_stop_ms()
        fl.sync()
        res.append(ms / args.steps if ms > 0 else None)
        del fl, out
    return res[0], res[1]


def ring_launch_roofline(plan, d_codes, outs, rows, err, n_batches=400):
    """The same batches through ONE launch (the resident ring, pgm_rows_ring_*: batch b = the rows and
    output buffers of resident batch b % len(outs)), after the timed region: the per-launch roofline of a
    single kernel instance — its duration from HIP events on its stream around the launch (start,
    posting of all n_batches, completion), which a rocprofv3 kernel trace of the same command reports as
    one `pgm_rows_ring` dispatch.  achieved = n_batches x the batch's algorithmic bytes / that duration."""
    import torch

    nb = len(outs)
    ring = plan.ring([(d_codes, rows * nb, i * rows, outs[i]) for i in range(nb)], rows, err=err)
    kname, k_blocks, k_wg = ring.kernel()
    # warm, same size (so a rocprofv3 --stats average over both dispatches is the timed one's duration):
    # the kernel's first-use load, every slot touched.  replay: 400 batches over the resident slots, whose
    # inputs never change (each repeat writes the same outputs)
    ring.run(n_batches, replay=True)
    torch.cuda.synchronize()
    timer = HipTimer()
    timer.start()
    ring.run(n_batches, replay=True)
    timer.mark_end()
    torch.cuda.synchronize()
    ms = timer.elapsed_ms()
    assert int(err.item()) == 0
    del ring
    nbytes = plan.algorithmic_bytes_per_row(marginals=True) * rows * n_batches
    achieved = nbytes / (ms * 1e-3) / 1e9
    return {"kernel": kname, "grid": {"blocks": k_blocks, "workgroup": k_wg}, "batches": n_batches,
            "rows_per_batch": rows, "launches": 1, "kernel_ms": ms, "ms_per_batch": ms / n_batches,
            "bytes_per_launch": nbytes, "achieved": achieved, "frac": achieved / HBM_PEAK_GBS,
            "slots": nb, "working_set_bytes": plan.algorithmic_bytes_per_row(marginals=True) * rows * nb,
            "working_set_over_mall": plan.algorithmic_bytes_per_row(marginals=True) * rows * nb / MALL_BYTES,
            "working_set_exceeds_mall": plan.algorithmic_bytes_per_row(marginals=True) * rows * nb > MALL_BYTES}


def hbm_stream_roofline(plan, d_codes, rows, nb, args, err, qs, n_out=24, steps=200):
    """The C3 launch streamed over n_out distinct output buffers (n_out x 13.6 MB > the 256 MiB MALL, so
    the outputs of a step are evicted to HBM before the buffer comes round again) on args.queues
    queues; inputs cycle over the nb resident batches (0.7 MB read per launch).  Average GPU span per
    launch over `steps` launches, outside the timed region; the bytes / span are an HBM rate."""
    import torch

    outs = [plan.alloc_outputs(rows, marginals=True) for _ in range(n_out)]
    bounds = [plan.bind(d_codes, rows * nb, (i % nb) * rows, rows, outs[i], err=err) for i in range(n_out)]
    q = max(1, args.queues)
    ln = Launcher(bounds, "direct", queues=min(q, n_out), qs=qs)
    ln.steps(n_out)
    ln.sync()
    ln.timer_start()
    ln.steps(steps)
    ms = ln.timer_stop_ms()
    ln.sync()
    same = all(torch.equal(outs[i]["marg"], outs[i % nb]["marg"]) for i in range(nb, n_out, 5))
    bpl = plan.algorithmic_bytes_per_row(marginals=True) * rows
    kms = ms / steps
    ach = bpl / (kms * 1e-3) / 1e9 if kms > 0 else None
    del ln, bounds, outs
    return {"output_buffers": n_out, "queues": min(q, n_out), "steps": steps,
            "working_set_bytes": bpl * n_out, "kernel_ms": kms, "achieved": ach,
            "frac": ach / HBM_PEAK_GBS if ach else None, "outputs_match_resident_batches": same}


def load_traffic(kernel):
    """HBM bytes/launch from a committed rocprofv3 PMC summary (profiles/pmc_<kernel>.json), if present."""
    path = os.path.join(ROOT, "profiles", f"pmc_{kernel}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), d.get("rows_per_launch")


def cpu_baseline_c3(model, missing, codes_host, nodes, seconds):
    """numpy oracle (oracle/ve.py), per-row predict_probability semantics, single core."""
    from oracle import ve as OVE
    from oracle.network import load_network

    net = load_network("munin")
    pos = {v: i for i, v in enumerate(nodes)}
    obs = [v for v in nodes if v not in missing]
    t0 = time.perf_counter()
    n = 0
    while True:
        ev = {v: net.states[v][codes_host[pos[v], n]] for v in obs}
        OVE.query(net, list(missing), ev, joint_out=False)
        n += 1
        if time.perf_counter() - t0 > seconds or n >= codes_host.shape[1]:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "queries/s", "cores": 1, "kind": "port",
            "sample": f"first {n} of the same synthetic munin rows, numpy oracle per-row query "
                      f"(prune + greedy einsum contraction + normalize + marginals), {dt:.1f} s"}


def _cpu_worker(job):
    """One host worker of the all-core CPU baseline: rows w, w+W, ... of the sample until the budget."""
    missing, codes_host, nodes, w, W, seconds = job
    from oracle import ve as OVE
    from oracle.network import load_network

    net = load_network("munin")
    pos = {v: i for i, v in enumerate(nodes)}
    obs = [v for v in nodes if v not in missing]
    t0 = time.perf_counter()
    n = 0
    for r in range(w, codes_host.shape[1], W):
        ev = {v: net.states[v][codes_host[pos[v], r]] for v in obs}
        OVE.query(net, list(missing), ev, joint_out=False)
        n += 1
        if time.perf_counter() - t0 > seconds:
            break
    return n


def cpu_baseline_c3_allcore(missing, codes_host, nodes, seconds):
    """The same oracle on every host core we are given (fork pool, before any GPU use)."""
    import multiprocessing as mp

    W = max(1, min(16, len(os.sched_getaffinity(0))))
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(W) as pool:
        counts = pool.map(_cpu_worker, [(list(missing), codes_host, nodes, w, W, seconds) for w in range(W)])
    dt = time.perf_counter() - t0
    return {"value": sum(counts) / dt, "unit": "queries/s", "cores": W, "kind": "port",
            "sample": f"{sum(counts)} rows of the same synthetic munin sample, numpy oracle per row, "
                      f"{W} worker processes, {dt:.1f} s wall (upper bound: pgmpy's predict is GIL-bound); "
                      f"W is capped at 16, the GPU box's CPU share per GPU (OMP_NUM_THREADS / MAX_JOBS there), "
                      f"not the {os.cpu_count()} CPUs the host shows",
            "cap_reason": "per-GPU CPU share of the box"}


def cpu_baselines_c3(args):
    """Both C3 CPU baselines, computed before the GPU is touched (the all-core pool forks)."""
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    model = get_example_model("munin")
    missing = set(random.Random(0).sample(sorted(model.nodes()), 3))
    codes_all, nodes = forward_sample_codes(model, args.rows, seed=42)
    single = cpu_baseline_c3(model, missing, codes_all, nodes, args.cpu_seconds)
    allcore = cpu_baseline_c3_allcore(missing, codes_all, nodes, min(10.0, args.cpu_seconds))
    return single, allcore


def api_e2e_rate(model, codes_all, nodes, missing, reps=5):
    """The shipped API on the same rows: DiscreteBayesianNetwork.predict_probability over a pandas
    Categorical DataFrame of the observed columns (host frame in, DataFrame out: ingestion, pattern
    grouping, the fused kernel, the result frame), best of `reps` after 3 warm calls (the first call of a
    frame schema validates every column's categories), outside the timed region (ADVICE r02:
    the line's `value` is the device-resident launch rate; this is what a DataFrame caller gets)."""
    import pandas as pd
    import torch

    st = model.states
    pos = {v: i for i, v in enumerate(nodes)}
    keep = [v for v in nodes if v not in missing]
    df = pd.DataFrame({c: pd.Categorical.from_codes(codes_all[pos[c]].astype(np.int8), categories=list(st[c]))
                       for c in keep})
    model.predict_probability(df.iloc[:1000])  # compile the pattern's plan
    for _ in range(3):  # warm calls: the frame's schema validated once, pinned result blocks cached
        model.predict_probability(df)
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        model.predict_probability(df)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    best = min(times)
    return {"value": len(df) / best, "unit": "rows/s", "rows": len(df), "seconds": best,
            "seconds_each": times, "median_rows_per_s": len(df) / float(np.median(times)),
            "path": "DiscreteBayesianNetwork.predict_probability(pandas Categorical frame) -> DataFrame"}


def parity_spot_check(model, missing, plan, out, codes_host, nodes, n_check=64, r0=0):
    """First rows of the device output (evidence columns r0.. of codes_host) against the oracle
    (1e-6 relative, BASELINE.json)."""
    from oracle import ve as OVE
    from oracle.network import load_network
    from pgmpy_amd.inference.batch import download

    net = load_network("munin")
    pos = {v: i for i, v in enumerate(nodes)}
    obs = [v for v in nodes if v not in missing]
    marg = download(out["marg"])
    worst = 0.0
    for r in range(n_check):
        ev = {v: net.states[v][codes_host[pos[v], r0 + r]] for v in obs}
        m = OVE.query(net, list(plan.variables), ev, joint_out=False)
        exp = np.concatenate([m[v] for v in plan.variables])
        got = marg[:, r]
        both_nan = np.isnan(exp) & np.isnan(got)
        err = np.abs(got - exp)[~both_nan] / np.maximum(np.abs(exp[~both_nan]), 1e-300)
        mask = np.abs(exp[~both_nan]) > 1e-12
        if mask.any():
            worst = max(worst, float(err[mask].max()))
    return {"rows_checked": n_check, "max_rel_err": worst, "ok": worst <= 1e-6}


def bench_c3(args, dist, rank, world):
    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    model = get_example_model("munin")
    missing_list = random.Random(0).sample(sorted(model.nodes()), 3)
    missing = set(model.nodes()) - (set(model.nodes()) - set(missing_list))
    variables = list(missing)  # the reference's predict_probability column order (set iteration)
    rows = args.rows
    nb = max(1, args.batches)  # distinct resident batches, stepped round robin
    t0 = time.perf_counter()
    codes_all, nodes = forward_sample_codes(model, rows, seed=42 + rank)
    observed = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    codes_one = np.ascontiguousarray(codes_all[[pos[v] for v in observed]])  # [1038, rows]
    # batch 0 = the sampled rows; batch i > 0 = a seeded row permutation of them (distinct inputs and
    # outputs per batch without re-running the sampler)
    prng = np.random.default_rng(1000 + rank)
    perms = [np.arange(rows)] + [prng.permutation(rows) for _ in range(nb - 1)]
    col_of = {v: i for i, v in enumerate(observed)}
    plan = PatternPlan(model, variables, observed, col_of)
    assert plan.kind == "fused", plan.describe()
    if nb > 1:  # [1038, rows * nb], filled in place (no list of copies: 96 batches are 10 GB)
        # every batch holds all 1,038 observed columns as stored; the columns the plan reads are the
        # batch's row permutation (its own evidence), the others a plain copy of the sampled rows
        # (never read by the pass, never used by the parity checks — they keep the as-stored layout
        # without a 10 GB fancy-index permutation per run)
        used = sorted({col_of[v] for v in plan.ev_used})
        codes_ev = np.empty((codes_one.shape[0], rows * nb), dtype=np.uint8)
        for i, p in enumerate(perms):
            codes_ev[:, i * rows:(i + 1) * rows] = codes_one
            if i:
                codes_ev[used, i * rows:(i + 1) * rows] = codes_one[used][:, p]
    else:
        codes_ev = codes_one
    del codes_one
    log(f"[rank {rank}] sampled {rows} rows, {nb} batch(es), in {time.perf_counter() - t0:.1f}s")
    d_codes = upload_codes(codes_ev)
    outs = [plan.alloc_outputs(rows, marginals=True) for _ in range(nb)]
    out = outs[0]
    err = torch.zeros(1, dtype=torch.int32, device=d_codes.device)
    # one step = one pass of the fused row plan over one resident batch (batch i = evidence columns
    # [i*rows, (i+1)*rows), its own output), launched through the prepared (bound) C-ABI entry:
    # validated and marshalled once, one argument-free call per step
    if args.launch == "ring":
        return bench_c3_ring(args, dist, rank, world, model, missing, variables, plan, d_codes, outs, err, codes_all,
                             nodes, perms)
    bounds = [plan.bind(d_codes, rows * nb, i * rows, rows, outs[i], err=err) for i in range(nb)]
    nq = args.queues if args.launch == "direct" else 1
    launcher = Launcher(bounds, args.launch, group=args.group, queues=nq)
    launcher.steps(max(args.warmup, nb))
    launcher.sync()
    if args.launch == "direct" and not args.acquire_in_window:
        # the first dispatch on a queue after a sync acquires at system scope (so inputs HIP wrote since
        # become visible); nothing writes the resident batches from here on, so one more untimed dispatch
        # per queue takes that acquire and the timed window holds steady-state dispatches only
        # (pgm_dq_wait: completion without a new release barrier, which would re-arm the acquire)
        launcher.steps(len(launcher.qs))
        launcher.wait()
    barrier(dist)
    # GPU span of the timed dispatches (queue timestamps or HIP events on the launch stream):
    # average launch duration, including the gap between back-to-back launches that rocprofv3's
    # kernel time omits
    launcher.timer_start()
    t_start = time.perf_counter()
    if args.release_mode == "launch":
        launcher.steps_released(args.steps)
    else:
        launcher.steps(args.steps)
    # the window closes on every step's dispatch complete AND its outputs visible system-wide: on the
    # direct queues the last launch of each queue releases at system scope on its own completion
    # (pgm_dq_launch_release), then every dispatch is waited for; HIP: the end event + torch.cuda.synchronize
    launcher.release_and_wait()
    t_end = time.perf_counter()
    kern_ms_total = launcher.timer_stop_ms()  # dispatch timestamps, read after the timed region
    barrier(dist)
    elapsed = max_over_ranks(dist, t_end - t_start)
    assert int(err.item()) == 0
    total_rows = rows * world * args.steps
    value = total_rows / elapsed
    kern_ms = kern_ms_total / args.steps
    if kern_ms <= 0:  # queue timestamps off (PGM_DQ_PROFILE=0): the wall time per step
        kern_ms = (t_end - t_start) * 1e3 / args.steps
    bpr = plan.algorithmic_bytes_per_row(marginals=True)
    achieved = bpr * rows / (kern_ms * 1e-3) / 1e9
    floor_ms, single_ms = dispatch_floor_ms(plan, d_codes, rows, args, Launcher)
    working_set = bpr * rows * nb
    stream = None
    if args.launch == "direct" and working_set <= MALL_BYTES:
        stream = hbm_stream_roofline(plan, d_codes, rows, nb, args, err, launcher.qs)
    ring_roof = None
    if not args.no_ring_roofline:
        try:
            ring_roof = ring_launch_roofline(plan, d_codes, outs, rows, err)
        except Exception as e:  # reported, never silently dropped; the headline above stands on its own
            ring_roof = {"error": f"{type(e).__name__}: {e}"}
    kname, k_blocks, k_wg = bounds[0].kernel()  # the kernel the bound launches run
    kname = kname or plan.kernel_name()
    traffic, traffic_rows = load_traffic(kname)
    if traffic is not None and traffic_rows:
        traffic = traffic * rows / traffic_rows
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (forward-sampled munin evidence rows, seed 42+rank)",
        "config": {
            "workload": "C3 munin predict_probability template: 3 missing / 1038 observed, "
                        "fused row plan (pgm_rows_plan_bind; one launch per step: one 100k-row batch, "
                        "batches resident in HBM and stepped round robin over the queues)",
            "launch": {"direct": "AQL packet on user-mode HSA queues (pgm_dq_launch; batch i on queue i % queues)",
                       "hip": "hipModuleLaunchKernel (pgm_rows_bound_run)"}[args.launch],
            "network": "munin",
            # what `value` measures: the fused row plan over evidence batches already resident in HBM
            # (prepared launch: kernel + dispatch); the public DataFrame API's end-to-end rate on the same
            # rows is `api_e2e` (host ingestion-bound)
            "value_measures": "device-resident evidence batches through the prepared fused-plan launch",
            "missing": variables,
            "rows_per_gpu_per_step": rows,
            "global_rows_per_step": rows * world,
            "batches": nb,
            "dispatch_group": args.group,
            "queues": nq,
            # each queue's first dispatch after the pre-window sync carries the system-scope acquire that
            # makes HIP-written inputs visible; it runs as an untimed warmup dispatch (the batches are not
            # written again), so the window's K dispatches all acquire nothing (--acquire-in-window: A/B)
            "acquire_before_window": args.launch == "direct" and not args.acquire_in_window,
            "parallelism": f"rows sharded over {world} GPU(s), no data-path collective",
            "plan": plan.describe(),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            # the same algorithmic bytes over the wall time per step of the timed window (dispatch,
            # completion and the closing system-scope release included): the rate `value` implies
            "frac_wall": bpr * rows * world / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS / world,
            "traffic": traffic,
            "kernel": kname,
            "kernel_ms": kern_ms,
            "grid": {"blocks": k_blocks, "workgroup": k_wg},
            # the same dispatch with the CPT staging and arithmetic removed (pgm_rows_floor[2]: same grid,
            # same code loads, same write-through output stores) and the kernel itself, each on one queue
            # after the timed region: what one launch of this shape costs before any inference work
            "dispatch_floor_ms": floor_ms,
            "single_queue_kernel_ms": single_ms,
            "kernel_over_floor": (single_ms / floor_ms) if floor_ms and single_ms else None,
            "algorithmic_bytes_per_row": bpr,
            "bytes_per_launch": bpr * rows,
            # kernel_ms is the GPU span per step; with Q queues up to Q launches run at once, so the
            # achieved rate is the launches' aggregate bytes over the span (a single dispatch's own
            # duration, rocprofv3's per-kernel time, is longer by up to the overlap)
            "concurrent_queues": nq,
            # the timed dispatches' own durations averaged (queue timestamps): the per-launch number to
            # compare with the committed rocprofv3 kernel-trace average (profiles/*_kernel_stats.csv)
            "dispatch_avg_ms": getattr(launcher, "dispatch_avg_ms", None),
            # every timed dispatch's own HSA timestamps ([queue, start, end] ticks at `freq` Hz): the span
            # above is max(end) - min(start) over them (tools/c3_span_check.py recomputes frac from these)
            "dispatch_times": getattr(launcher, "dispatch_times", None),
            # the batches' outputs + inputs (algorithmic bytes): the default 24 batches (343 MB) exceed
            # the MI355X's 256 MiB Infinity Cache (MALL), so a step's output lines are evicted to HBM
            # before its buffer comes round again and the achieved rate is an HBM rate; with a set
            # that fits (--batches <= 17) hbm_stream repeats the measurement over 24 output buffers
            "working_set_bytes": working_set,
            "working_set_over_mall": working_set / MALL_BYTES,
            "working_set_exceeds_mall": working_set > MALL_BYTES,
            "hbm_stream": stream,
            # per-launch roofline of ONE kernel instance over the same batches (resident ring, 400
            # batches, after the timed region): a duration a rocprofv3 kernel trace reproduces directly
            # (one dispatch), unlike the overlapped four-queue span above
            "single_launch_ring": ring_roof,
        },
    }
    if rank == 0:
        n_chk = max(16, 64 // nb)
        checks = [parity_spot_check(model, missing, plan, outs[i], codes_all[:, perms[i][:n_chk]], nodes,
                                    n_check=n_chk) for i in range(nb)]
        result["parity"] = {"rows_checked": sum(c["rows_checked"] for c in checks),
                            "batches_checked": nb,
                            "max_rel_err": max(c["max_rel_err"] for c in checks),
                            "ok": all(c["ok"] for c in checks)}
        if world == 1 and args.cpu_pre is not None:
            result["cpu_baseline"], result["cpu_baseline_allcore"] = args.cpu_pre
            result["cpu_baseline"]["cores_on_host"] = os.cpu_count()
        if world == 1 and not args.no_api_e2e:
            result["api_e2e"] = api_e2e_rate(model, codes_all, nodes, missing)
    if not args.no_c5:
        result["c5"] = c5_subline(args, dist, rank, world, model, variables, observed, plan, codes_ev, d_codes,
                                  rows * nb)
    if dist is not None:
        # the result delivery (outside the timed region in this weak-scaling line; --workload c5
        # times it inside the step): every rank's [17, rows] marginals to rank 0
        from pgmpy_amd.distributed import gather_rows

        barrier(dist)
        g0 = time.perf_counter()
        src = out["marg"] if _BACKEND == "nccl" else out["marg"].cpu()
        gather_rows(src, rows * world, dist)
        torch.cuda.synchronize()
        result["gather_ms"] = (time.perf_counter() - g0) * 1e3
        result["gather_backend"] = _BACKEND
    return result


def host_dma_probe(nbytes=136_000_000, reps=8):
    """How much device-to-host DMA one GPU's host link takes with one and with two concurrent streams
    (each stream its own pinned host buffer and device source): the ceiling C5's host delivery runs at
    per rank (Multi-GPU).  GB/s = bytes copied / wall time of all copies."""
    import torch

    from pgmpy_amd import _native as N

    n = nbytes // 8
    src = [torch.ones(n, dtype=torch.float64, device="cuda") for _ in range(2)]
    dst = [torch.empty(n, dtype=torch.float64, pin_memory=True) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    L = N.lib()

    def copy(i, nb):
        N.check(L.pgm_memcpy_d2h_async(ctypes.c_void_p(dst[i].data_ptr()), N.ptr(src[i]), nb,
                                       N.stream_handle(streams[i])), "memcpy_d2h_async")

    def run(n_streams, nb):
        for i in range(n_streams):
            copy(i, nb)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            for i in range(n_streams):
                copy(i, nb)
        torch.cuda.synchronize()
        return n_streams * nb * reps / (time.perf_counter() - t0) / 1e9

    one = run(1, n * 8)
    two_split = run(2, n * 4)  # the same bytes split over two streams
    two_full = run(2, n * 8)   # twice the bytes, one full copy per stream
    ok = bool(dst[0][:4].sum().item() == 4.0)
    del src, dst
    return {"bytes_per_copy": n * 8, "reps": reps, "one_stream_GBps": one, "two_streams_split_GBps": two_split,
            "two_streams_full_GBps": two_full, "copies_checked": ok}


def c5_subline(args, dist, rank, world, model, variables, observed, plan, codes_host, d_codes, ld):
    """BASELINE.json configs[4] inside the default line: 1 M rows per step split
    over the N ranks (strong scaling), each rank's block taken from its C3 resident rows (batch 0 and
    its seeded permutations), timed three ways after the C3 window: delivered to pinned host memory per
    rank (predict_probability's marginals, and predict's MAP indices), and gathered to rank 0 over
    RCCL (bench_c5).  Every rank runs it (collectives inside); rank 0's dict is reported."""
    import copy

    from pgmpy_amd.distributed import shard_bounds

    total = 1_000_000
    lo, hi = shard_bounds(total, world, rank)
    rows5 = hi - lo
    if rows5 > ld:
        return {"skipped": f"{rows5} rows per rank exceed the {ld} resident C3 rows"}
    inp = {"model": model, "variables": variables, "observed": observed, "plan": plan, "codes_host": codes_host,
           "d_codes": d_codes, "ld": ld, "rows": rows5, "total": total,
           "data": "synthetic (rank r's C3 resident rows: forward-sampled with seed 42+r and seeded row "
                   "permutations of them)"}
    out = {"workload": "C5 (BASELINE.json configs[4]): munin predict_probability / predict template, 1M rows per "
                       "step split over the ranks (strong scaling)",
           "global_rows_per_step": total, "rows_per_gpu_per_step": rows5, "n_gpus": world}
    keep = ("value", "unit", "ms_per_step", "steps", "kernel_ms", "copy_ms", "copy_bytes_per_rank", "copy_GBps",
            "pipelined_step_over_copy", "gather_ms", "launch_ms", "gather_backend", "gather_bytes_to_rank0",
            "roofline", "parity")
    for name, fn, output in (("host", bench_c5_host, "marginals"), ("host_map", bench_c5_host, "map"),
                             ("rccl", bench_c5, "marginals")):
        a = copy.copy(args)
        a.rows, a.c5_output = total, output
        try:
            r = fn(a, dist, rank, world, inp=inp)
            out[name] = {k: r[k] for k in keep if k in r}
            out[name]["delivery"] = r["config"].get("delivery", "rccl" if fn is bench_c5 else "host")
        except Exception as e:  # reported, never silently dropped; the headline stands on its own
            out[name] = {"error": f"{type(e).__name__}: {e}"}
    out["value"] = out["host"].get("value")
    if rank == 0:
        out["host_dma_probe"] = host_dma_probe()
    return out


def bench_c3_ring(args, dist, rank, world, model, missing, variables, plan, d_codes, outs, err, codes_all, nodes,
                  perms):
    """C3 through the resident ring (--launch ring, pgm_rows_ring_*): the K timed steps are K batches
    posted one by one to ONE launch of the plan-specialised kernel that is started inside the timed
    window.  Batch i runs the rows and output buffers of resident batch i % nb.  The window closes when
    the launch has completed (hipStreamSynchronize: HIP's end-of-kernel system-scope release included).
    The launch's own GPU span is bracketed by HIP events on its stream (kernel_ms = span / K); a
    rocprofv3 kernel trace reports the same launch ("pgm_rows_ring", one dispatch per timed region)."""
    import copy

    import torch

    rows = args.rows
    nb = len(outs)
    ring = plan.ring([(d_codes, rows * nb, i * rows, outs[i]) for i in range(nb)], rows, err=err)
    kname, k_blocks, k_wg = ring.kernel()
    ring.run(max(args.warmup, nb))  # every slot once
    torch.cuda.synchronize()
    timer = HipTimer()
    barrier(dist)
    launch_ms = None
    if args.ring_prestart:
        # the resident kernel is launched before the window, as a serving engine's would be before
        # requests arrive; the window holds the K batches' posts, their processing, the kernel's exit
        # and the closing synchronize (HIP's end-of-kernel system-scope release).  start returns once
        # every workgroup is resident with its CPT staged (pgm_rows_ring_start_ready), so the window
        # holds no part of the launch
        t_l = time.perf_counter()
        timer.start()
        ring.start(args.steps, wait_ready=True)
        timer.mark_end()
        launch_ms = (time.perf_counter() - t_l) * 1e3
        t_start = time.perf_counter()
    else:
        t_start = time.perf_counter()
        timer.start()
        ring.start(args.steps)
        timer.mark_end()  # the end event completes with the launch
    for b in range(1, args.steps + 1):
        ring.post(b)  # one step = one batch published to the resident launch
    ring.finish()
    t_end = time.perf_counter()
    kern_ms = timer.elapsed_ms() / args.steps
    barrier(dist)
    elapsed = max_over_ranks(dist, t_end - t_start)
    assert int(err.item()) == 0
    bpr = plan.algorithmic_bytes_per_row(marginals=True)
    achieved = bpr * rows / (kern_ms * 1e-3) / 1e9
    ms_per_step = elapsed * 1e3 / args.steps
    hip_args = copy.copy(args)
    hip_args.launch = "hip"
    floor_ms, single_ms = dispatch_floor_ms(plan, d_codes, rows, hip_args, Launcher)
    traffic, traffic_rows = load_traffic(kname)
    if traffic is not None and traffic_rows:
        traffic = traffic * rows / traffic_rows
    working_set = bpr * rows * nb
    result = {
        "metric": METRIC,
        "value": rows * world * args.steps / elapsed,
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (forward-sampled munin evidence rows, seed 42+rank)",
        "config": {
            "workload": "C3 munin predict_probability template: 3 missing / 1038 observed, fused row plan; "
                        "one step = one 100k-row batch posted to the resident ring launch (pgm_rows_ring_*), "
                        "batches resident in HBM, batch i on buffer set i % batches",
            "launch": ("one resident launch per timed region, launched and resident (every workgroup running) "
                       "before the window (--ring-prestart), K batches posted inside it" if args.ring_prestart else
                       "one resident launch per timed region (started inside the window), K batches posted"),
            "ring_host_launch_ms": launch_ms,
            "network": "munin",
            # what `value` measures: the fused row plan over evidence batches already resident in HBM
            # (prepared launch: kernel + dispatch); the public DataFrame API's end-to-end rate on the same
            # rows is `api_e2e` (host ingestion-bound)
            "value_measures": "device-resident evidence batches through the prepared fused-plan launch",
            "missing": variables,
            "rows_per_gpu_per_step": rows,
            "global_rows_per_step": rows * world,
            "batches": nb,
            "parallelism": f"rows sharded over {world} GPU(s), no data-path collective",
            "plan": plan.describe(),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            # the same algorithmic bytes over the driver-visible wall time per step (window includes
            # the launch, the posts and the closing synchronize)
            "frac_wall": bpr * rows / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": kname,
            "kernel_ms": kern_ms,
            "kernel_span_ms": kern_ms * args.steps,
            "grid": {"blocks": k_blocks, "workgroup": k_wg},
            "dispatch_floor_ms": floor_ms,
            "single_launch_kernel_ms": single_ms,
            "algorithmic_bytes_per_row": bpr,
            "bytes_per_launch": bpr * rows * args.steps,
            "bytes_per_step": bpr * rows,
            "working_set_bytes": working_set,
            "working_set_over_mall": working_set / MALL_BYTES,
            "working_set_exceeds_mall": working_set > MALL_BYTES,
        },
    }
    if rank == 0:
        n_chk = max(16, 64 // nb)
        checks = [parity_spot_check(model, missing, plan, outs[i], codes_all[:, perms[i][:n_chk]], nodes,
                                    n_check=n_chk) for i in range(nb)]
        result["parity"] = {"rows_checked": sum(c["rows_checked"] for c in checks), "batches_checked": nb,
                            "max_rel_err": max(c["max_rel_err"] for c in checks),
                            "ok": all(c["ok"] for c in checks)}
        if world == 1 and args.cpu_pre is not None:
            result["cpu_baseline"], result["cpu_baseline_allcore"] = args.cpu_pre
            result["cpu_baseline"]["cores_on_host"] = os.cpu_count()
        if world == 1 and not args.no_api_e2e:
            result["api_e2e"] = api_e2e_rate(model, codes_all, nodes, missing)
    del ring
    return result


def c5_inputs(args, rank, world):
    """C5's own inputs (--workload c5): rank r's contiguous block of the 1 M rows, forward-sampled with
    seed (42, first row of the block), all 1,038 observed columns resident on the device."""
    from pgmpy_amd.distributed import shard_bounds
    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    model = get_example_model("munin")
    missing_list = random.Random(0).sample(sorted(model.nodes()), 3)
    variables = list(set(missing_list))
    total = args.rows
    lo, hi = shard_bounds(total, world, rank)
    rows = hi - lo
    t0 = time.perf_counter()
    codes_all, nodes = forward_sample_codes(model, rows, seed=(42, lo))
    observed = [v for v in nodes if v not in set(variables)]
    pos = {v: i for i, v in enumerate(nodes)}
    codes_ev = np.ascontiguousarray(codes_all[[pos[v] for v in observed]])
    del codes_all
    log(f"[rank {rank}] rows [{lo}, {hi}) sampled in {time.perf_counter() - t0:.1f}s")
    plan = PatternPlan(model, variables, observed, {v: i for i, v in enumerate(observed)})
    assert plan.kind == "fused", plan.describe()
    return {"model": model, "variables": variables, "observed": observed, "plan": plan, "codes_host": codes_ev,
            "d_codes": upload_codes(codes_ev), "ld": rows, "rows": rows, "total": total,
            "data": "synthetic (forward-sampled munin evidence rows, seed (42, first row of the block))"}


def rotating_roofline(plan, codes_host, rows, want_map, err, steps, min_over_mall=4.2):
    """Per-launch roofline of the fused pass at `rows` rows with an HBM-sized working set: nb batches,
    each its own compact evidence columns (the plan's used columns, batch i a seeded row permutation of
    codes_host's first `rows` rows) and its own output buffer, nb x (bytes per launch) >= min_over_mall x
    the 256 MiB Infinity Cache; back-to-back launches on one stream rotate over them, so no launch finds
    its outputs or inputs still in the MALL.  kernel_ms = HIP-event span / launches (a rocprofv3 kernel
    trace of the same command reports each launch)."""
    import math

    import torch

    from pgmpy_amd.inference.batch import upload_codes

    cp = plan.compact()
    bpr = plan.algorithmic_bytes_per_row(marginals=not want_map, map_=want_map)
    nb = max(2, math.ceil(min_over_mall * MALL_BYTES / (bpr * rows)))
    used = codes_host[[plan.col_of[v] for v in plan.ev_used], :rows]
    prng = np.random.default_rng(2025)
    host = np.empty((used.shape[0], rows * nb), dtype=np.uint8)
    for i in range(nb):
        host[:, i * rows:(i + 1) * rows] = used if i == 0 else used[:, prng.permutation(rows)]
    d = upload_codes(host)
    outs = [cp.alloc_outputs(rows, marginals=not want_map, map_=want_map) for _ in range(nb)]
    st = torch.cuda.Stream(device=d.device)
    bounds = [cp.bind(d, rows * nb, i * rows, rows, outs[i], err=err, stream=st) for i in range(nb)]
    n_launch = max(steps, 2 * nb)
    with torch.cuda.stream(st):
        for b in bounds:  # first use: every buffer touched once
            b.run()
        timer = HipTimer()
        timer.start()
        for j in range(n_launch):
            bounds[j % nb].run()
        timer.mark_end()
    torch.cuda.synchronize()
    ms = timer.elapsed_ms() / n_launch
    assert int(err.item()) == 0
    kname, k_blocks, k_wg = bounds[0].kernel()
    del bounds, outs, d
    ws = bpr * rows * nb
    achieved = bpr * rows / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": kname,
            "grid": {"blocks": k_blocks, "workgroup": k_wg}, "kernel_ms": ms, "launches": n_launch,
            "algorithmic_bytes_per_row": bpr, "bytes_per_launch": bpr * rows, "rotating_batches": nb,
            "working_set_bytes": ws, "working_set_over_mall": ws / MALL_BYTES,
            "working_set_exceeds_mall": ws > MALL_BYTES,
            "kernel_ms_note": "HIP-event span / launches of back-to-back launches on one stream, each batch its "
                              "own compact evidence columns and output buffer, rotating (outside the window)"}


def bench_c5_host(args, dist, rank, world, inp=None):
    """C5 delivered to host memory (the default, --c5-delivery host): every rank writes its block's
    results into pinned host memory of its node over its OWN host link, with no collective — the
    result of predict_probability / predict is a host DataFrame, and a funnel into one GPU (the RCCL
    gather, --c5-delivery rccl) moves every row's 136 B through rank 0's links.  One step = each
    rank's fused-plan launch over its block (device-resident evidence) into device buffer k % 2 +
    the DMA of that buffer into pinned host buffer k % 2, ordered as HostDelivery's mode says (default
    "lanes": launch k and copy k on stream lane k % 2, so copy k overlaps launch k + 1).
    `inp` (c5_inputs' dict) lets the default C3 line run this step on its own resident rows."""
    import torch

    from pgmpy_amd.distributed import HostDelivery

    inp = inp or c5_inputs(args, rank, world)
    plan, variables, observed = inp["plan"], inp["variables"], inp["observed"]
    d_codes, ld, rows, total, codes_ev = inp["d_codes"], inp["ld"], inp["rows"], inp["total"], inp["codes_host"]
    dev = d_codes.device
    want_map = args.c5_output == "map"
    key = "map" if want_map else "marg"
    outs = [plan.alloc_outputs(rows, marginals=not want_map, map_=want_map) for _ in range(2)]
    delivery = HostDelivery(tuple(outs[0][key].shape), outs[0][key].dtype, depth=2, device=dev)
    hosts = delivery.hosts
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    ls = torch.cuda.Stream(device=dev)
    bounds = [plan.bind(d_codes, ld, 0, rows, outs[i], err=err, stream=delivery.launch_stream(i, ls))
              for i in range(2)]

    def step(k):
        s = delivery.launch_stream(k, ls)
        delivery.acquire(k, s)  # device buffer k % 2 and host slot k % 2 are free
        bounds[k % 2].run()
        delivery.deliver(k, outs[k % 2][key], s)

    for k in range(max(args.warmup, 2)):
        step(k)
    torch.cuda.synchronize()
    barrier(dist)
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(k)
    delivery.wait()
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    barrier(dist)
    elapsed = max_over_ranks(dist, t_end - t_start)
    assert int(err.item()) == 0
    # the parts alone, outside the window: the launch over rotating HBM-sized buffers (the roofline),
    # and the copy-out (back to back, one stream)
    roof = rotating_roofline(plan, codes_ev, rows, want_map, err, args.steps)
    kernel_ms = roof["kernel_ms"]
    t0 = time.perf_counter()
    with torch.cuda.stream(ls):
        for k in range(args.steps):
            hosts[k % 2].copy_(outs[k % 2][key], non_blocking=True)
    ls.synchronize()
    copy_ms = (time.perf_counter() - t0) * 1e3 / args.steps
    copy_bytes = hosts[0].numel() * hosts[0].element_size()
    parity = None
    if rank == 0:
        from oracle import ve as OVE  # checker only: first rows of rank 0's block, from the HOST copy
        from oracle.network import load_network

        net = load_network("munin")
        got = hosts[(args.steps - 1) % 2].numpy()
        worst, wrong, checked = 0.0, 0, 0
        for r in range(min(rows, 16)):
            ev = {v: net.states[v][codes_ev[j, r]] for j, v in enumerate(observed)}
            if want_map:
                mp, gap = OVE.map_query(net, list(plan.variables), ev)
                if gap <= 1e-9:
                    continue
                flat = 0
                for v in plan.variables:
                    flat = flat * len(net.states[v]) + net.states[v].index(mp[v])
                wrong += int(got[r] != flat)
            else:
                m = OVE.query(net, variables, ev, joint_out=False)
                exp = np.concatenate([m[v] for v in plan.variables])
                worst = max(worst, float(np.max(np.abs(got[:, r] - exp) / np.maximum(np.abs(exp), 1e-300))))
            checked += 1
        parity = ({"rows_checked": checked, "map_mismatches": wrong, "ok": wrong == 0} if want_map else
                  {"rows_checked": checked, "max_rel_err": worst, "ok": worst <= 1e-6, "checked_on": "host copy"})
    ms_per_step = elapsed * 1e3 / args.steps
    roof["step_bound"] = "host link (PCIe D2H of the block's results)"
    return {
        "metric": METRIC, "value": total * args.steps / elapsed, "unit": "queries/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": inp["data"],
        "config": {"workload": ("C5 munin predict (MAP) template, 1M rows per step sharded over the ranks, "
                                "int32 MAP indices delivered to pinned host memory per rank") if want_map else
                               ("C5 munin predict_probability template, 1M rows per step sharded over the ranks, "
                                "marginals delivered to pinned host memory per rank"),
                   "network": "munin", "missing": variables, "global_rows_per_step": total,
                   "rows_per_gpu_per_step": rows, "delivery": "host",
                   "launch": f"bound fused-plan launch into device buffer k % 2, DMA to pinned host buffer k % 2, "
                             f"HostDelivery mode {delivery.mode!r}",
                   "parallelism": f"rows sharded over {world} rank(s), no collective: each rank's own host link"},
        "kernel_ms": kernel_ms, "copy_ms": copy_ms, "copy_bytes_per_rank": copy_bytes,
        "copy_GBps": copy_bytes / (copy_ms * 1e-3) / 1e9,
        "pipelined_step_over_copy": ms_per_step / copy_ms if copy_ms else None,
        "roofline": roof,
        "parity": parity,
    }


def bench_c5(args, dist, rank, world, inp=None):
    """C5 (BASELINE.json configs[4]) with the RCCL funnel (--c5-delivery rccl): ROWS (1,000,000) munin
    template rows per step over all ranks, contiguous blocks per rank (distributed.shard_bounds),
    strong scaling.  One step = every rank's bound fused-plan launch over its block + the gather of the
    [17, rows] fp64 marginals to rank 0 (torch.distributed.gather: RCCL over xGMI with the nccl
    backend).  Rank 0 owns a [world, 17, block] receive buffer allocated once; blocks are padded to the
    largest so one gather serves all.  `inp`: see bench_c5_host."""
    import torch

    from pgmpy_amd.distributed import shard_bounds

    inp = inp or c5_inputs(args, rank, world)
    plan, variables, observed = inp["plan"], inp["variables"], inp["observed"]
    d_codes, ld, rows, total, codes_ev = inp["d_codes"], inp["ld"], inp["rows"], inp["total"], inp["codes_host"]
    block = max(h - l for l, h in (shard_bounds(total, world, r) for r in range(world)))
    dev = d_codes.device
    want_map = getattr(args, "c5_output", "marginals") == "map"
    # three output buffers on three streams: step k's launch writes buffer k % 3 on stream k % 3
    # while step k-1's buffer is gathered on its own stream (the gather of step k-1 is issued right
    # after launch k, so the collective overlaps the next launch).  At N = 1 the three marginal
    # buffers are 3 x 136 MB > the 256 MiB Infinity Cache, so every step's outputs reach HBM.
    nbuf = 3
    sends, outs = [], []
    for _ in range(nbuf):
        if want_map:  # predict(): the MAP assignment per row, as the plan's int32 flat index
            send = torch.zeros((1, block), dtype=torch.int32, device=dev)
            outs.append({"map": send[0, :rows] if rows else send[0, :1]})
        else:  # predict_probability(): the [17, rows] marginals, ld = block (padded)
            send = torch.zeros((plan.n_acc, block), dtype=torch.float64, device=dev)
            outs.append({"marg": send[:, :rows] if rows else send[:, :1]})
        sends.append(send)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(nbuf)]
    torch.cuda.synchronize()
    bounds = [plan.bind(d_codes, ld, 0, rows, outs[i], err=err, stream=streams[i]) for i in range(nbuf)]
    nccl = dist is not None and _BACKEND == "nccl"
    recvs = [None] * nbuf
    if dist is not None and rank == 0:
        recvs = [[torch.empty(tuple(sends[0].shape), dtype=sends[0].dtype, device=dev if nccl else "cpu")
                  for _ in range(world)] for _ in range(nbuf)]
    host_send = None if nccl or dist is None else torch.empty(tuple(sends[0].shape), dtype=sends[0].dtype)

    def launch(k):
        bounds[k % nbuf].run()  # on stream k % 2: after that stream's previous gather

    def gather(k):
        """step k's results to rank 0, ordered after step k's launch (same stream); later work on
        that stream (launch k + 2) waits for the collective."""
        if dist is None:
            return
        i = k % nbuf
        with torch.cuda.stream(streams[i]):
            if nccl:
                dist.gather(sends[i], gather_list=recvs[i], dst=0)
            else:  # gloo rehearsal: through host memory
                streams[i].synchronize()
                host_send.copy_(sends[i])
                dist.gather(host_send, gather_list=recvs[i], dst=0)

    def run_steps(k0, n):
        for k in range(k0, k0 + n):
            launch(k)
            if k > k0:
                gather(k - 1)
        gather(k0 + n - 1)

    run_steps(0, max(args.warmup, nbuf))
    torch.cuda.synchronize()
    barrier(dist)
    t_start = time.perf_counter()
    run_steps(0, args.steps)  # every step's launch and its gather inside the window
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    barrier(dist)
    elapsed = max_over_ranks(dist, t_end - t_start)
    assert int(err.item()) == 0
    # the launches alone, then the gathers alone, outside the timed region (wall per step, max over ranks)
    barrier(dist)
    l0 = time.perf_counter()
    for k in range(args.steps):
        launch(k)
    torch.cuda.synchronize()
    launch_ms = max_over_ranks(dist, (time.perf_counter() - l0) * 1e3 / args.steps)
    # one launch's own duration: the same launches one after another on one stream (HIP events)
    seq = [plan.bind(d_codes, ld, 0, rows, outs[i], err=err, stream=streams[0]) for i in range(nbuf)]
    with torch.cuda.stream(streams[0]):
        timer = HipTimer()
        timer.start()
        for k in range(args.steps):
            seq[k % nbuf].run()
        kernel_ms = timer.stop_ms() / args.steps
    torch.cuda.synchronize()
    del seq
    barrier(dist)
    g0 = time.perf_counter()
    for k in range(args.steps):
        gather(k)
    torch.cuda.synchronize()
    gather_ms = max_over_ranks(dist, (time.perf_counter() - g0) * 1e3 / args.steps)
    bpr = plan.algorithmic_bytes_per_row(marginals=not want_map, map_=want_map)
    roof = rotating_roofline(plan, codes_ev, rows, want_map, err, args.steps)
    parity = None
    if rank == 0:
        from oracle import ve as OVE  # checker only: first rows of rank 0's block
        from oracle.network import load_network
        from pgmpy_amd.inference.batch import download

        net = load_network("munin")
        got = download(sends[(args.steps - 1) % nbuf][:, :min(rows, 16)].contiguous())
        worst, wrong, checked = 0.0, 0, 0
        for r in range(got.shape[1]):
            ev = {v: net.states[v][codes_ev[j, r]] for j, v in enumerate(observed)}
            if want_map:
                mp, gap = OVE.map_query(net, list(plan.variables), ev)
                if gap <= 1e-9:
                    continue  # a near-tie may break either way
                flat = 0
                for v in plan.variables:
                    flat = flat * len(net.states[v]) + net.states[v].index(mp[v])
                wrong += int(got[0, r] != flat)
                checked += 1
            else:
                m = OVE.query(net, variables, ev, joint_out=False)
                exp = np.concatenate([m[v] for v in plan.variables])
                worst = max(worst, float(np.max(np.abs(got[:, r] - exp) / np.maximum(np.abs(exp), 1e-300))))
                checked += 1
        if dist is not None and nccl and not want_map:  # rank 0's gathered copy of its own block
            same = torch.equal(recvs[(args.steps - 1) % nbuf][0], sends[(args.steps - 1) % nbuf])
            parity_gather = bool(same)
        else:
            parity_gather = None
        parity = ({"rows_checked": checked, "map_mismatches": wrong, "ok": wrong == 0} if want_map else
                  {"rows_checked": checked, "max_rel_err": worst, "ok": worst <= 1e-6,
                   "gathered_equals_local": parity_gather})
    ms_per_step = elapsed * 1e3 / args.steps
    return {
        "metric": METRIC,
        "value": total * args.steps / elapsed,
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": inp["data"],
        "config": {"workload": ("C5 munin predict (MAP) template, 1M rows per step sharded over the ranks + gather "
                                "of the int32 MAP indices to rank 0") if want_map else
                               ("C5 munin predict_probability template, 1M rows per step sharded over the ranks "
                                "+ gather of the marginals to rank 0"),
                   "network": "munin", "missing": variables, "global_rows_per_step": total,
                   "launch": "hipModuleLaunchKernel (bound), three streams / three output buffers, gather of "
                             "step k-1 issued after launch k",
                   "rows_per_gpu_per_step": rows, "parallelism": f"rows sharded over {world} rank(s), "
                   f"{_BACKEND if dist is not None else 'no'} gather to rank 0"},
        "gather_ms": gather_ms if dist is not None else 0.0,
        "launch_ms": launch_ms,
        "gather_backend": _BACKEND if dist is not None else None,
        "gather_bytes_to_rank0": (8 if not want_map else 4) * (plan.n_acc if not want_map else 1) * block * (world - 1),
        "roofline": dict(roof, frac_wall=bpr * rows / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         three_buffer_kernel_ms=kernel_ms),
        "parity": parity,
    }


def bench_c2(args):
    """C2: one munin query, 100 leaf findings -> 1 root, greedy device contraction.  The evidence rows
    are the reference's own (tests/golden/munin_c2_rows.json: forward_sample(size=20, seed=0) of
    pgmpy, the same 100 findings per row, so one compiled plan): step k queries row k % 20.  After the
    timed region every row is checked against the reference on two outputs of the SAME compiled
    program: the root posterior (one-hot on all 20 rows, so it pins the support) and the unnormalised
    joint before normalize, P(root, findings) over the pruned model (1e-46 .. 1e-28: it pins the scale;
    ExactInference.py:404-420, make_golden.py gen_munin_c2_mass) at rtol 1e-9."""
    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    with open(os.path.join(ROOT, "tests", "golden", "munin_c2_rows.json")) as f:
        g = json.load(f)
    m = get_example_model("munin")
    q = g["variables"]
    rows = [r["evidence"] for r in g["rows"]]
    ve = VariableElimination(m)
    torch.cuda.synchronize()
    t_cold = time.perf_counter()
    ve.query(q, rows[0], show_progress=False)  # first query of the pattern: prune, plan, compile, capture
    torch.cuda.synchronize()
    t_cold = time.perf_counter() - t_cold
    for k in range(args.warmup):
        ve.query(q, rows[k % len(rows)], show_progress=False)
    gc.collect()  # compile-time objects collected before the window (see bench_c1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        r = ve.query(q, rows[k % len(rows)], show_progress=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    runner, = ve._compiled.values()
    plan = runner.plan
    ps = plan.path_stats(1)
    prog = plan.__dict__.get("_q1", {}).get("joint", (None,))[0]
    worst, worst_mass, ok = 0.0, 0.0, True
    masses = []
    for row, ev in zip(g["rows"], rows):
        got = ve.query(q, ev, show_progress=False)
        want = np.asarray(row["root"]["values"], dtype=np.float64)
        x = np.asarray(got.values).ravel()
        ok &= bool(np.allclose(x, want, rtol=1e-6, atol=1e-12))
        worst = max(worst, float(np.max(np.abs(x - want))))
        un = np.asarray(ve.query_unnormalized(q, ev).values, dtype=np.float64).ravel()
        want_un = np.asarray(row["root_unnormalized"], dtype=np.float64)
        ok &= bool(np.allclose(un, want_un, rtol=1e-9, atol=0))
        worst_mass = max(worst_mass, float(np.max(np.abs(un - want_un)) / np.max(np.abs(want_un))))
        masses.append(float(want_un.sum()))
    ok &= len(ve._compiled) == 1  # the checked outputs came from the timed program
    out = {"metric": "munin single-row query latency (C2)", "value": dt, "unit": "s/query",
           "higher_is_better": False, "steps": args.steps, "warmup": args.warmup, "first_query_s": t_cold,
           "plan": {"kind": plan.kind, **ps},
           "launches_per_query": len(prog._direct) if prog is not None and prog._direct else None,
           "dispatch": getattr(prog, "direct_note", None),
           "roofline": {"bound": "latency (dependent launches; the executed plan's bytes take ~8 us at HBM peak)",
                        "achieved": ps["bytes"] / dt / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ps["bytes"] / dt / 1e9 / HBM_PEAK_GBS, "traffic": None,
                        "tflops": ps["flops"] / dt / 1e12,
                        "note": "algorithmic bytes / flops of the executed plan (contraction.choose_path; "
                                "SURVEY §8(d) C2) per query over the wall time per query"},
           "reference": {"value": float(np.mean([r["seconds"][-1] for r in g["rows"]])), "unit": "s/query",
                         "note": "pgmpy's own VariableElimination.query on these 20 rows (opt_einsum shim, greedy; "
                                 "make_golden.py gen_munin_c2_mass, 5 processes on the build container's 8-core "
                                 "Xeon) - not this host"},
           "note": "steady state: the evidence pattern's compiled plan is cached (new evidence values, "
                   "same query/evidence variables); first_query_s includes pruning, planning and compiling",
           "data": "the reference's 20 forward-sampled munin rows (tests/golden/munin_c2_rows.json), step k = row k % 20",
           "parity": {"ok": ok, "rows_checked": len(rows), "max_abs_err": worst, "rtol": 1e-6, "atol": 1e-12,
                      "mass_max_rel_err": worst_mass, "mass_rtol": 1e-9,
                      "mass_range": [min(masses), max(masses)],
                      "against": "reference root posteriors AND unnormalised root joints (tests/golden/munin_c2_rows.json), "
                                 "both read from the timed program's outputs"},
           "result": list(np.asarray(r.values))}
    if not args.no_cpu_baseline:
        # the oracle's prune + classic elimination (oracle.ve.eliminate: the build's elimination rule in
        # numpy; its greedy_contract restates opt_einsum's greedy, which takes ~46 s per query here like
        # the reference) on all 20 rows, one core
        from oracle import ve as OVE
        from oracle.network import load_network

        net = load_network("munin")
        t0 = time.perf_counter()
        for ev in rows:
            OVE.query(net, q, ev, contract=OVE.eliminate)
        out["cpu_baseline"] = {"value": (time.perf_counter() - t0) / len(rows), "unit": "s/query", "cores": 1,
                               "kind": "port", "sample": "the same 20 rows, numpy oracle: pruning + classic "
                                                         "variable elimination in min-clique order (oracle.ve.eliminate)"}
    return out


def bench_c1(args):
    """C1: alarm VariableElimination.query, single evidence rows: the reference's own 50 seeded patterns
    (tests/golden/alarm_queries.json, SURVEY §8(d) C1: 3 query variables, 5 findings from
    forward_sample(seed=1)), device path (compiled per pattern), every pattern's joint checked against
    the reference after the timed region; the numpy oracle on the host beside it."""
    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    with open(os.path.join(ROOT, "tests", "golden", "alarm_queries.json")) as f:
        g = json.load(f)
    pats = [(p["variables"], p["evidence"]) for p in g["patterns"]]
    m = get_example_model("alarm")
    ve = VariableElimination(m)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for q, e in pats:
        ve.query(q, e, show_progress=False)
    torch.cuda.synchronize()
    cold = (time.perf_counter() - t0) / len(pats)
    # the 50 plans' compile-time objects are collected now, not by a full collection inside the window
    # (a one-time ~50 ms pause that landed in 300-step windows and not in 200-step ones: 0.078 vs 0.044 ms)
    gc.collect()
    t0 = time.perf_counter()
    reps = max(1, args.steps // 10)
    for _ in range(reps):
        for q, e in pats:
            ve.query(q, e, show_progress=False)
    torch.cuda.synchronize()
    warm = (time.perf_counter() - t0) / (reps * len(pats))
    worst, ok = 0.0, True
    for p in g["patterns"]:
        r = ve.query(p["variables"], p["evidence"], show_progress=False)
        got = np.asarray(r.values, dtype=np.float64).ravel()
        want = np.asarray(p["joint"]["values"], dtype=np.float64)
        ok &= list(r.variables) == list(p["joint"]["variables"]) and bool(np.allclose(got, want, rtol=1e-6, atol=1e-12))
        worst = max(worst, float(np.max(np.abs(got - want))))
    h = g["history_cvp_low"]
    r = ve.query(["HISTORY"], {"CVP": "LOW"}, show_progress=False)
    ok &= bool(np.allclose(np.asarray(r.values).ravel(), h["values"], rtol=1e-6, atol=1e-12))
    direct = sum(bool(getattr(h_[0], "_direct", None)) for rn in ve._compiled.values()
                 for h_ in rn.plan.__dict__.get("_q1", {}).values())
    out = {"metric": "alarm single-row query latency (C1)", "value": warm, "unit": "s/query",
           "higher_is_better": False, "patterns": len(pats), "queries_timed": reps * len(pats),
           "first_query_s": cold, "programs_on_aql_chain": direct,
           "roofline": {"bound": "latency (a few dependent launches per query; bytes are a few KB)",
                        "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None, "traffic": None},
           "note": "value: compiled pattern plans cached (same query/evidence variables, new values)",
           "parity": {"ok": ok, "patterns_checked": len(pats) + 1, "max_abs_err": worst, "rtol": 1e-6,
                      "atol": 1e-12, "against": "reference joints (tests/golden/alarm_queries.json) + "
                                                "HISTORY|CVP=LOW"}}
    if not args.no_cpu_baseline:
        from oracle import ve as OVE
        from oracle.network import load_network

        net = load_network("alarm")
        t0, n = time.perf_counter(), 0
        while n < len(pats) or time.perf_counter() - t0 < 2.0:
            q, e = pats[n % len(pats)]
            OVE.query(net, q, e)
            n += 1
        out["cpu_baseline"] = {"value": (time.perf_counter() - t0) / n, "unit": "s/query", "cores": 1,
                               "kind": "port", "sample": f"{n} queries over the same 50 patterns, numpy oracle "
                                                         "(pruning + greedy contraction per call)"}
    # the oracle is a readable restatement (it re-prunes per call and contracts with plain einsum), not a
    # stand-in for pgmpy's speed here: the reference's own latency on C1 is quoted beside it
    out["reference"] = {"value": 0.43e-3, "unit": "s/query",
                        "note": "pgmpy VariableElimination.query(['HISTORY'], {'CVP': 'LOW'}), greedy, median of 20, "
                                "survey container (8-core Xeon; BASELINE.md) - not this host"}
    return out


def _c4_pmc_summary():
    """The committed PMC summary of the C4 sweep (tools/c4_step_pmc.py: separate FETCH_SIZE / WRITE_SIZE
    rocprofv3 passes over one 4,000-row replay, FETCH x2 per the MI355X guide): the newest round's."""
    import glob

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*", "c4pmc_summary.json")),
                   key=lambda p: (os.path.basename(os.path.dirname(p))[:3], os.path.getmtime(p)))
    if not paths:
        return None
    with open(paths[-1]) as f:
        d = json.load(f)
    return {"source": os.path.relpath(paths[-1], ROOT), "rows": d.get("rows"),
            "fetch_bytes_x2": d.get("fetch_bytes_x2"), "write_bytes": d.get("write_bytes"),
            "hbm_side_bytes": d.get("hbm_side_bytes"), "floor_bytes": d.get("floor_bytes"),
            "ratio_to_floor": d.get("ratio_to_floor"), "ratio_to_step_bytes": d.get("ratio_to_step_bytes")}


def bench_c4(args):
    """C4: pathfinder batched BP calibration (min-fill JT), 4 leaf findings per row.  value: one
    calibration batch at a time (BatchedJunctionTree inflight=1, what BeliefPropagation.calibrate_batch
    runs by default); `two_in_flight` the same batches with two in flight (calibrate_batch(inflight=2))."""
    import torch

    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.inference.EliminationOrder import junction_tree_from_model
    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import leaf_findings_codes

    m = get_example_model("pathfinder")
    jt = junction_tree_from_model(m)
    bjt = BatchedJunctionTree(jt, inflight=1)
    n = args.rows
    ev, ev_vars, _, _ = leaf_findings_codes(m, n, per_row=4, seed=7)
    d = upload_codes(ev)

    def rate(inflight):
        bjt.inflight, bjt._lane = inflight, 0
        for _ in range(max(1, args.warmup) * inflight):
            bjt.calibrate_codes(d, ev_vars, n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            c = bjt.calibrate_codes(d, ev_vars, n)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps, c

    dt, cal = rate(1)
    two = None
    if args.c4_inflight > 1:  # lane 0's compiled schedule is shared with the one-at-a-time run
        dt2, _ = rate(args.c4_inflight)
        two = {"value": n / dt2, "unit": "calibrations/s", "inflight": args.c4_inflight, "ms_per_step": dt2 * 1e3,
               "note": "the same calibration batches with this many in flight (own schedules and streams, "
                       "round robin; BeliefPropagation.calibrate_batch(inflight=k))"}
        bjt.inflight, bjt._lane = 1, 0
    bpc = bjt.bytes_per_calibration()
    sch = bjt.schedule(n, ev_vars, "marginalize", False)
    parity = _c4_parity(m, cal, ev, ev_vars, n)
    step_bytes = sum(sch.prog.step_bytes) / n if sch.prog.step_bytes else None
    out = {"metric": "pathfinder BP calibrations/s (C4)", "value": n / dt, "unit": "calibrations/s",
           "higher_is_better": True, "rows_per_step": n, "steps": args.steps, "ms_per_step": dt * 1e3,
           "inflight": 1,
           "roofline": {"bound": "hbm", "achieved": bpc * n / dt / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": bpc * n / dt / 1e9 / HBM_PEAK_GBS, "traffic": None,
                        "bytes_per_calibration": bpc,
                        "executed_step_bytes_per_calibration": step_bytes,
                        "executed_step_GBps": step_bytes * n / dt / 1e9 if step_bytes else None,
                        "executed_step_frac": step_bytes * n / dt / 1e9 / HBM_PEAK_GBS if step_bytes else None,
                        "pmc": _c4_pmc_summary(),
                        "note": "achieved: this schedule's floor (every belief written once, every separator "
                                "message / sigma' written and read once: 8 (sum|C| + 4 sum|S|)) over the wall time "
                                "per calibration; executed_step_bytes: every tensor each launched step reads or "
                                "writes; pmc: memory-side bytes of one 4,000-row replay (committed rocprofv3 "
                                "passes) against that floor"},
           "reference_schedule_bytes_per_calibration": bjt.reference_bytes_per_calibration(),
           "reference_schedule_note": "SURVEY §8(d) C4's 8 (4 sum|C| + 4 sum|S|) counts every belief read and "
                                      "written in both passes; this schedule does not move those bytes, so that "
                                      "figure over this rate is not an achieved bandwidth",
           "cliques": len(bjt.cliques),
           "two_in_flight": two,
           "parity": parity}
    if not args.no_cpu_baseline:
        # the oracle's calibration (oracle/bp.py: findings as 0/1 indicators, one collect + one
        # distribute sweep of _update_beliefs) row by row for ~10 s, one core
        from oracle import bp as OBP
        from oracle.network import load_network
        from pgmpy_amd.inference.EliminationOrder import min_fill_decomposition

        net = load_network("pathfinder")
        bags, edges = min_fill_decomposition(m)
        pots = OBP.initial_potentials(net, bags)
        t0, done = time.perf_counter(), 0
        while done < n and (done < 2 or time.perf_counter() - t0 < args.cpu_seconds_c4):
            r = done
            e = {v: net.states[v][int(ev[j, r])] for j, v in enumerate(ev_vars) if ev[j, r] != 255}
            OBP.calibrate(bags, edges, OBP.apply_evidence(net, pots, bags, e))
            done += 1
        out["cpu_baseline"] = {"value": done / (time.perf_counter() - t0), "unit": "calibrations/s", "cores": 1,
                               "kind": "port", "sample": f"the first {done} rows of the same batch, numpy oracle "
                                                         "(oracle/bp.py calibrate), one row at a time"}
    out["reference"] = {"value": 1 / 1.8, "unit": "calibrations/s",
                        "note": "pgmpy BeliefPropagation(jt).calibrate() on this junction tree, 1.66-1.96 s, survey "
                                "container (SURVEY §6) - not this host"}
    return out


def _c4_parity(m, cal, ev, ev_vars, n):
    """After the timed region: 16 rows of the last timed calibration (first, last, 14 seeded), every
    entry of every clique belief against the oracle's calibration of the row's findings (the checker;
    tests/test_inference_gpu.py::test_pathfinder_c4_bench_schedule runs 32 rows)."""
    from oracle import bp as OBP
    from oracle.network import load_network
    from pgmpy_amd.inference.EliminationOrder import min_fill_decomposition

    rows = sorted({0, n - 1} | set(int(x) for x in np.random.default_rng(11).choice(n, min(n, 14), replace=False)))
    bags, edges = min_fill_decomposition(m)
    try:
        worst, entries = OBP.check_batched_rows(load_network("pathfinder"), bags, edges,
                                                cal.clique_beliefs_rows(rows), ev, ev_vars, rows, rtol=1e-9)
        return {"ok": True, "rows_checked": len(rows), "entries": entries, "max_rel_err": worst, "rtol": 1e-9,
                "oracle": "oracle/bp.py (pinned to tests/golden/pathfinder_bp.*)"}
    except AssertionError as e:
        return {"ok": False, "rows_checked": len(rows), "error": str(e)[:400]}


def subconfigs(args):
    """BASELINE.json configs[0], [1] and [3] as sub-objects of the default (C3) line at N = 1, each run
    after the C3 window with its own timing, roofline, parity and same-host one-core CPU baseline
    (the driver's own run measures them).  Step counts are fixed here so the line's
    total stays a few minutes whatever --steps the driver passes."""
    import copy

    import torch

    out = {}
    for name, fn, over in (("c1", bench_c1, dict(steps=100, warmup=5)),
                           ("c2", bench_c2, dict(steps=400, warmup=40)),
                           ("c4", bench_c4, dict(steps=20, warmup=3, rows=4000))):
        a = copy.copy(args)
        vars(a).update(over)
        t0 = time.perf_counter()
        try:
            out[name] = fn(a)
        except Exception as e:  # reported, never silently dropped; the headline stands on its own
            out[name] = {"error": f"{type(e).__name__}: {e}"}
        out[name]["bench_s"] = round(time.perf_counter() - t0, 2)
        gc.collect()
        torch.cuda.empty_cache()
        log(f"[sub] {name} {out[name].get('value')} ({out[name]['bench_s']} s)")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rows", type=int, default=None,
                    help="c3: rows per GPU per step (100,000); c5: rows per step over all GPUs (1,000,000)")
    ap.add_argument("--workload", default="c3", choices=["c3", "c5", "c1", "c2", "c4"])
    ap.add_argument("--c5-output", default="marginals", choices=["marginals", "map"],
                    help="c5: gather the fp64 marginals (predict_probability) or the MAP indices (predict)")
    ap.add_argument("--c5-delivery", default="host", choices=["host", "rccl"],
                    help="c5: each rank DMAs its block's results into pinned host memory (host, no collective) "
                         "or gathers them into rank 0's GPU over RCCL (rccl)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c4-inflight", type=int, default=2,
                    help="c4: also time this many calibration batches in flight (own schedules, own streams, "
                         "round robin; the headline is one at a time)")
    ap.add_argument("--cpu-seconds-c4", type=float, default=10.0, help="c4: seconds of oracle calibrations")
    ap.add_argument("--no-subconfigs", action="store_true",
                    help="c3 at N=1: skip the c1 / c2 / c4 sub-objects (configs[0], [1], [3])")
    ap.add_argument("--no-api-e2e", action="store_true", help="c3: skip the public-API DataFrame rate")
    ap.add_argument("--no-c5", action="store_true",
                    help="c3: skip the C5 sub-object (1M rows split over the ranks: host delivery, MAP, RCCL gather)")
    ap.add_argument("--no-ring-roofline", action="store_true",
                    help="c3: skip the single-launch (resident ring) roofline after the timed region")
    ap.add_argument("--release-mode", default="barrier", choices=["launch", "barrier"],
                    help="c3 direct: the window's system-scope release on the last launch per queue (launch) or as "
                         "one barrier packet per queue appended together (barrier)")
    ap.add_argument("--ring-prestart", action="store_true",
                    help="c3 --launch ring: launch the resident kernel just before the timed window")
    ap.add_argument("--gather", action="store_true", help="c3: after timing, gather marginals to rank 0 (RCCL)")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"])
    ap.add_argument("--batches", type=int, default=96,
                    help="c3: distinct resident row batches (each its own evidence columns and output), "
                         "stepped round robin; 96 x 14.3 MB = 1.37 GB = 5.1x the 256 MiB Infinity Cache, so "
                         "a batch's output lines are evicted to HBM long before its buffer comes round again")
    ap.add_argument("--group", type=int, default=1,
                    help="c3 direct launch: dispatch this many consecutive steps (distinct batches) as one "
                         "pgm_dq_launch_group (<= --batches)")
    ap.add_argument("--queues", type=int, default=4,
                    help="c3 direct launch: spread the batches over this many user-mode HSA queues "
                         "(batch i on queue i %% Q; <= --batches)")
    ap.add_argument("--acquire-in-window", action="store_true",
                    help="c3 (A/B): leave each queue's first system-scope acquire inside the timed window")
    ap.add_argument("--launch", default="direct", choices=["direct", "hip", "ring"],
                    help="c3/c5: AQL packets on a user-mode HSA queue (direct), hipModuleLaunchKernel (hip); "
                         "c3: batches posted to one resident launch (ring)")
    args = ap.parse_args()
    if args.rows is None:
        args.rows = {"c3": 100_000, "c5": 1_000_000}.get(args.workload, 1000)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    from pgmpy_amd.build import build

    build(verbose=False)
    args.cpu_pre = None
    single_process = int(os.environ.get("WORLD_SIZE", "1")) == 1
    if args.workload == "c3" and single_process and not args.no_cpu_baseline:
        args.cpu_pre = cpu_baselines_c3(args)  # before dist_setup: no GPU state in the forked workers
    dist, rank, world = dist_setup(args.gpus, args.dist_backend)
    if args.workload == "c3":
        res = bench_c3(args, dist, rank, world)
        if world == 1 and not args.no_subconfigs:
            res.update(subconfigs(args))
    elif args.workload == "c5":
        res = (bench_c5_host if args.c5_delivery == "host" else bench_c5)(args, dist, rank, world)
    elif args.workload == "c2":
        res = bench_c2(args)
    elif args.workload == "c1":
        res = bench_c1(args)
    else:
        res = bench_c4(args)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
