"""Multi-rank evidence sharding with world_size 2 on CPU (gloo).

The CPU test's per-rank executor is the numpy oracle (test infrastructure): it
checks the host logic of pgmpy_amd.distributed — contiguous row blocks, the
single gather to rank 0 and the reassembly order — not the kernels (those are
covered by the -m gpu tests).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from pgmpy_amd.distributed import shard_bounds


def test_shard_bounds_cover_rows():
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            sizes = [hi - lo for lo, hi in b]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_rows, result_path):
    import torch
    import torch.distributed as dist

    from oracle import ve as OVE
    from oracle.network import load_network
    from pgmpy_amd.distributed import run_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    net = load_network("alarm")
    rng = np.random.default_rng(0)
    ev_vars = ["CVP", "PCWP", "HISTORY"]
    codes = np.stack([rng.integers(0, net.card[v], n_rows) for v in ev_vars]).astype(np.uint8)
    q = ["LVFAILURE", "HYPOVOLEMIA"]

    def executor(block, row_offset):
        out = []
        for r in range(block.shape[1]):
            ev = {v: net.states[v][int(block[j, r])] for j, v in enumerate(ev_vars)}
            m = OVE.query(net, q, ev, joint_out=False)
            out.append(np.concatenate([m[v] for v in q]))
        return torch.tensor(np.array(out).T.copy())  # [n_marg, rows], rows innermost

    got = run_sharded(executor, codes, n_rows, dist)
    if rank == 0:
        np.save(result_path, got.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gather_matches_single_rank(tmp_path):
    from oracle import ve as OVE
    from oracle.network import load_network

    n_rows = 37
    path = str(tmp_path / "gathered.npy")
    mp.spawn(_worker, args=(2, _free_port(), n_rows, path), nprocs=2, join=True)
    got = np.load(path)
    net = load_network("alarm")
    rng = np.random.default_rng(0)
    ev_vars = ["CVP", "PCWP", "HISTORY"]
    codes = np.stack([rng.integers(0, net.card[v], n_rows) for v in ev_vars]).astype(np.uint8)
    q = ["LVFAILURE", "HYPOVOLEMIA"]
    for r in range(n_rows):
        ev = {v: net.states[v][int(codes[j, r])] for j, v in enumerate(ev_vars)}
        m = OVE.query(net, q, ev, joint_out=False)
        np.testing.assert_allclose(got[:, r], np.concatenate([m[v] for v in q]), atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_hip_predict_matches_golden(tmp_path, world):
    """The sharded HIP path of C5 (BASELINE.json configs[4]) at world 2 and 3 (uneven blocks):
    each rank runs the bound fused row plan on its block of the 2,000 reference munin rows, the
    [17, rows] marginals and MAP indices are gathered to rank 0; the gathered result must equal
    the single-launch run bit for bit and the reference fixture (marginals 1e-6 relative, MAP
    exact).  With a GPU per rank the gather is RCCL (world 1 on the one-GPU box: a one-rank RCCL
    communicator, so the nccl backend really executes); ranks sharing one card use gloo."""
    import subprocess
    import sys

    from tests.goldens import munin_predict

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / "sharded.npz")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(root, "tests", "workers", "sharded_predict.py"), out]
    r = subprocess.run(cmd, cwd=root, timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    z = np.load(out)
    assert int(z["world"]) == world
    if world == 1:
        assert str(z["backend"]) == "nccl"
    np.testing.assert_array_equal(z["sharded_marg"], z["full_marg"])
    np.testing.assert_array_equal(z["sharded_map"], z["full_map"])
    g = munin_predict()
    prob = z["full_marg"].T  # [rows, 17] in the fixture's column order
    np.testing.assert_allclose(prob, g["prob"], rtol=1e-6, atol=1e-300)
    cards = [int(c) for c in z["cards"]]
    idx = z["full_map"].copy()
    digits = {}
    for v, c in reversed(list(zip(z["variables"], cards))):
        digits[str(v)] = idx % c
        idx //= c
    got = np.stack([digits[v] for v in g["missing"]], axis=1)
    np.testing.assert_array_equal(got, g["map_codes"])


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2])
def test_sharded_host_delivery_matches_golden(tmp_path, world):
    """C5's default delivery (bench.py --c5-delivery host): no gather — every rank DMAs its block's
    marginals and MAP indices into pinned host memory through pgmpy_amd.distributed.HostDelivery
    (double-buffered, copies overlapping the next launch); the blocks, reassembled in rank order, equal
    the reference fixture's 2,000 rows (marginals 1e-6 relative, MAP exact).  World 2 on the one-GPU box:
    two ranks sharing the card (gloo process group, no collective on the data path)."""
    import subprocess
    import sys

    from tests.goldens import munin_predict

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / "host")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(root, "tests", "workers", "sharded_predict.py"), out, "host"]
    r = subprocess.run(cmd, cwd=root, timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    parts = [np.load(f"{out}.rank{k}.npz") for k in range(world)]
    assert [int(p["lo"]) for p in parts] == sorted(int(p["lo"]) for p in parts)
    assert int(parts[0]["lo"]) == 0 and all(int(a["hi"]) == int(b["lo"]) for a, b in zip(parts, parts[1:]))
    marg = np.concatenate([p["marg"] for p in parts], axis=1)
    mp = np.concatenate([p["map"] for p in parts])
    g = munin_predict()
    assert marg.shape[1] == g["codes"].shape[1] == int(parts[-1]["hi"])
    np.testing.assert_allclose(marg.T, g["prob"], rtol=1e-6, atol=1e-300)
    digits = {}
    for v, c in reversed(list(zip(parts[0]["variables"], [int(c) for c in parts[0]["cards"]]))):
        digits[str(v)] = mp % c
        mp = mp // c
    np.testing.assert_array_equal(np.stack([digits[v] for v in g["missing"]], axis=1), g["map_codes"])
