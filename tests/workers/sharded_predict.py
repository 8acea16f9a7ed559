"""Rank worker for tests/test_distributed.py::test_sharded_hip_predict_matches_golden (-m gpu).

Launched as `python -m torch.distributed.run --nproc-per-node N tests/workers/sharded_predict.py OUT`.
Every rank runs the HIP fused row plan (bound launch, as bench.py --workload c5) on its contiguous
block of the 2,000 reference munin template rows (tests/golden/munin_predict.npz), the marginals and
MAP indices are gathered to rank 0 (nccl = RCCL when every rank has its own GPU, else gloo through
host memory), and rank 0 also runs all rows in one launch and saves both for the test to compare.
With a third argument "host" no result is gathered: every rank delivers its block's marginals and MAP
indices into pinned host memory (pgmpy_amd.distributed.HostDelivery, the C5 default of bench.py) and
saves them to OUT.rank<r>.npz with its row bounds; the test reassembles the blocks.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(out_path, mode="gather"):
    import torch
    import torch.distributed as dist

    from goldens import munin_predict, prob_var_order
    from pgmpy_amd.distributed import gather_rows, shard_bounds
    from pgmpy_amd.inference.batch import download, upload_codes
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    n_dev = torch.cuda.device_count()
    dev = local % n_dev
    torch.cuda.set_device(dev)
    nccl = n_dev >= world
    if nccl:
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group("gloo")

    g = munin_predict()
    model = get_example_model("munin")
    observed = list(g["columns"])
    variables = prob_var_order(g["prob_columns"], g["missing"], model.states)
    plan = PatternPlan(model, variables, observed, {v: i for i, v in enumerate(observed)})
    assert plan.kind == "fused", plan.describe()
    codes = np.ascontiguousarray(g["codes"], dtype=np.uint8)  # [1038, 2000]
    n = codes.shape[1]
    lo, hi = shard_bounds(n, world, rank)

    def run(block):
        m = block.shape[1]
        d = upload_codes(block)
        out = plan.alloc_outputs(m, marginals=True, map_=True)
        err = torch.zeros(1, dtype=torch.int32, device=d.device)
        plan.bind(d, m, 0, m, out, err=err).run()
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        return out

    if mode == "host":
        from pgmpy_amd.distributed import HostDelivery

        block = np.ascontiguousarray(codes[:, lo:hi])
        m = block.shape[1]
        d = upload_codes(block)
        outs = [plan.alloc_outputs(m, marginals=True, map_=True) for _ in range(2)]
        err = torch.zeros(1, dtype=torch.int32, device=d.device)
        ls = torch.cuda.Stream()
        dm = HostDelivery(tuple(outs[0]["marg"].shape), torch.float64, device=d.device)
        dp = HostDelivery(tuple(outs[0]["map"].shape), torch.int32, device=d.device, lanes=dm.lanes)
        bounds = [plan.bind(d, m, 0, m, o, err=err, stream=dm.launch_stream(i, ls)) for i, o in enumerate(outs)]
        for k in range(5):  # consecutive steps through the double buffers, copies overlapping launches
            s = dm.launch_stream(k, ls)
            dm.acquire(k, s)
            dp.acquire(k, s)
            bounds[k % 2].run()
            dm.deliver(k, outs[k % 2]["marg"], s)
            dp.deliver(k, outs[k % 2]["map"], s)
        hm, hp = dm.wait(4), dp.wait(4)
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        np.savez(f"{out_path}.rank{rank}.npz", lo=lo, hi=hi, marg=hm.numpy(), map=hp.numpy().astype(np.int64),
                 backend="nccl" if nccl else "gloo", variables=np.array(variables), cards=np.array(plan.cards))
        dist.barrier()
        dist.destroy_process_group()
        return
    mine = run(np.ascontiguousarray(codes[:, lo:hi]))
    marg = mine["marg"] if nccl else mine["marg"].cpu()
    mp = mine["map"].to(torch.int64)
    mp = (mp if nccl else mp.cpu()).reshape(1, -1)
    gm = gather_rows(marg, n, dist)
    gp = gather_rows(mp, n, dist)
    if rank == 0:
        full = run(codes)
        np.savez(out_path, world=world, backend="nccl" if nccl else "gloo",
                 sharded_marg=gm.cpu().numpy(), sharded_map=gp.cpu().numpy().reshape(-1),
                 full_marg=download(full["marg"]), full_map=download(full["map"]).astype(np.int64),
                 variables=np.array(variables), cards=np.array(plan.cards))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(*sys.argv[1:3])
