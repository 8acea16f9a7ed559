#!/usr/bin/env python3
"""Dump the C4 schedule (pathfinder, ROWS rows, default 4,000): per step its level, full note,
algorithmic bytes, time when replayed alone, and the generated source of every specialised step.

    python3 tools/c4_dump.py OUT_DIR

Writes OUT_DIR/steps.json and OUT_DIR/step_<i>.hip (specialised steps only)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _time_bound(L, N, h, reps=20):
    """us per launch of one bound specialised step, replayed alone on the current stream."""
    import torch

    s = N.stream_handle()
    N.check(L.pgm_pm_bound_run(h, s), "pm_bound_run")
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    N.check(L.pgm_event_create(ctypes.byref(a)))
    N.check(L.pgm_event_create(ctypes.byref(b)))
    N.check(L.pgm_event_record(a, s))
    for _ in range(reps):
        N.check(L.pgm_pm_bound_run(h, s), "pm_bound_run")
    N.check(L.pgm_event_record(b, s))
    torch.cuda.synchronize()
    ms = ctypes.c_float()
    N.check(L.pgm_event_elapsed_ms(a, b, ctypes.byref(ms)))
    L.pgm_event_destroy(a)
    L.pgm_event_destroy(b)
    return ms.value * 1e3 / reps


def main():
    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.inference.EliminationOrder import junction_tree_from_model
    from pgmpy_amd.utils import get_example_model

    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    rows = int(os.environ.get("ROWS", "4000"))
    m = get_example_model("pathfinder")
    bjt = BatchedJunctionTree(junction_tree_from_model(m))
    leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)
    sch = bjt.schedule(rows, leaves, graph=False, marginals=False)
    prog = sch.prog
    prog.run()
    torch.cuda.synchronize()
    times = prog.time_steps()
    L = N.lib()
    buf = ctypes.create_string_buffer(1 << 22)
    pm = {h.value for h in prog._pm_bound}  # specialised handles (batch handles are not)
    steps = []
    for i, (fn, (us, note)) in enumerate(zip(prog._steps, times)):
        rec = {"i": i, "level": prog.step_levels[i] if i < len(prog.step_levels) else None, "us": us,
               "MB": prog.step_bytes[i] / 1e6 if i < len(prog.step_bytes) else None, "note": note,
               "parts": prog.merged_parts.get(i)}
        hs = prog.merged_handles.get(i)
        if hs and os.environ.get("PARTS", "1") == "1":  # each merged step alone, unmerged
            arr = (ctypes.c_void_p * len(hs))(*[h.value for h in hs])
            N.check(L.pgm_pm_prepare(arr, len(hs)), "pm_prepare")
            rec["part_us"] = [_time_bound(L, N, h) for h in hs]
        bs = getattr(fn, "bounds", ())
        b = bs[0] if len(bs) == 1 else None
        if isinstance(b, ctypes.c_void_p) and b.value in pm:
            n = L.pgm_pm_bound_source(b, buf, len(buf))
            if n > 0:
                with open(os.path.join(out, f"step_{i}.hip"), "w") as f:
                    f.write(buf.value.decode())
                rec["source"] = f"step_{i}.hip"
        steps.append(rec)
    json.dump({"rows": rows, "total_us": sum(s["us"] for s in steps), "steps": steps,
               "cliques": {str(c): bjt.sizes[c] for c in bjt.cliques}, "root": str(bjt.root)},
              open(os.path.join(out, "steps.json"), "w"), indent=1)
    print("steps", len(steps), "sum of step times", round(sum(s["us"] for s in steps), 1), "us")


if __name__ == "__main__":
    main()
