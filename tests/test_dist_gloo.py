"""Multi-process path on CPU (gloo, world_size 2): scenario sharding by global
id + the end-of-batch all-gather reproduce the single-process batch exactly.
The per-rank compute here is the C oracle (this container has no GPU); on the
GPU box the same dist.py functions carry the HIP results over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out_path):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root), str(root / "mpc-ntm-control_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ntm_mpc.dist import gather_scenarios, shard_range
    from oracle import cbind
    from oracle import ntm_oracle as O
    first, count = shard_range(total, world, rank)
    x0 = O.scenario_x0(np.arange(first, first + count)).T
    cfg = O.Config(N=3, mode=2)
    res = cbind.run(x0, cfg, 4, nthreads=1)
    uk = gather_scenarios(torch.from_numpy(res["uk"]), total)
    xk = gather_scenarios(torch.from_numpy(res["xk"]), total)
    fl = gather_scenarios(torch.from_numpy(res["exitflag"]), total)
    from ntm_mpc.dist import gather_to_root
    roots = {k: gather_to_root(torch.from_numpy(np.ascontiguousarray(res[k])), total)
             for k in ("uk", "Uk", "xk", "wpred", "exitflag", "inner_iters")}
    if rank != 0:
        assert all(v is None for v in roots.values())
    if rank == 0:
        np.savez(out_path, uk=uk.numpy(), xk=xk.numpy(), fl=fl.numpy(),
                 **{"root_" + k: v.numpy() for k, v in roots.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 13), (2, 8), (3, 10)])
def test_sharded_gather_equals_single_process(tmp_path, world, total):
    out = tmp_path / "g.npz"
    mp.spawn(_worker, args=(world, _free_port(), total, str(out)), nprocs=world, join=True)
    g = np.load(out)
    from oracle import cbind
    from oracle import ntm_oracle as O
    ref = cbind.run(O.scenario_x0(np.arange(total)).T, O.Config(N=3, mode=2), 4, nthreads=1)
    np.testing.assert_array_equal(g["uk"], ref["uk"])        # bitwise: scenarios are independent
    np.testing.assert_array_equal(g["xk"], ref["xk"])
    np.testing.assert_array_equal(g["fl"], ref["exitflag"])
    for k in ("uk", "Uk", "xk", "wpred", "exitflag", "inner_iters"):          # gather to rank 0 only
        np.testing.assert_array_equal(g["root_" + k], ref[k], err_msg=k)


def test_shard_range_partitions():
    from ntm_mpc.dist import shard_range
    for total in (0, 1, 7, 100000, 800000):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(c for _, c in spans) == total
            for (f0, c0), (f1, _) in zip(spans, spans[1:]):
                assert f0 + c0 == f1
