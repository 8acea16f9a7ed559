"""Where the fixed cost of a short timed region goes (direct AQL launch of the C3 bound plan):
host time of K launches, wait for the last dispatch, torch.cuda.synchronize() on an idle device,
single-dispatch round trip.  Prints one JSON line."""
import json
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    torch.cuda.set_device(0)
    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    rows = 100_000
    codes, nodes = forward_sample_codes(m, rows, seed=42)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    plan = PatternPlan(m, list(set(missing)), obs, {v: i for i, v in enumerate(obs)})
    d = upload_codes(np.ascontiguousarray(codes[[pos[v] for v in obs]]))
    out = plan.alloc_outputs(rows, marginals=True)
    direct = plan.bind(d, rows, 0, rows, out).direct()
    q = direct.queue
    for _ in range(20):
        direct.run()
    q.sync()
    torch.cuda.synchronize()
    res = {}
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res["torch_sync_idle_us"] = float(np.median(ts) * 1e6)
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        q.sync()
        ts.append(time.perf_counter() - t0)
    res["dq_sync_idle_us"] = float(np.median(ts) * 1e6)
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        direct.run()
        q.sync()
        ts.append(time.perf_counter() - t0)
    res["one_dispatch_roundtrip_us"] = float(np.median(ts) * 1e6)
    br = []
    for _ in range(50):
        q.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            direct.run()
        t1 = time.perf_counter()
        q.timer_start()  # (not bracketing: only to keep the API exercised)
        q.sync()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        q.timer_stop_ms()
        br.append((t1 - t0, t2 - t1, t3 - t2))
    br = np.median(np.array(br), axis=0) * 1e6
    res["k20_launch_host_us"], res["k20_wait_last_us"], res["k20_torch_sync_us"] = map(float, br)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
