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
    from ntm_mpc.dist import gather_scenarios, gather_to_root, shard_range
    from oracle import cbind
    from oracle import ntm_oracle as O
    first, count = shard_range(total, world, rank)
    x0 = O.scenario_x0(np.arange(first, first + count)).T
    cfg = O.Config(N=3, mode=2)
    res = cbind.run(x0, cfg, 4, nthreads=1)
    uk = gather_scenarios(torch.from_numpy(res["uk"]), total)
    xk = gather_scenarios(torch.from_numpy(res["xk"]), total)
    fl = gather_scenarios(torch.from_numpy(res["exitflag"]), total)
    roots = {k: gather_to_root(torch.from_numpy(np.ascontiguousarray(res[k])), total)
             for k in ("uk", "Uk", "xk", "wpred", "exitflag", "inner_iters")}
    if rank != 0:
        assert all(v is None for v in roots.values())
    # a subgroup without global rank 0: root is group-relative (its rank 0 is global rank 1)
    sub_ranks = list(range(1, world))
    sub = dist.new_group(sub_ranks) if world > 2 else None
    sub_uk = None
    if sub is not None and rank in sub_ranks:
        st = sum(shard_range(total, world, r)[1] for r in sub_ranks)
        sub_uk = gather_to_root(torch.from_numpy(np.ascontiguousarray(res["uk"])), st, root=0, group=sub)
        assert (sub_uk is not None) == (rank == 1)
        if rank == 1:
            np.save(str(out_path) + ".sub.npy", sub_uk.numpy())
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
    if world > 2:                                   # subgroup of ranks 1.., root group-relative
        from ntm_mpc.dist import shard_range
        first = shard_range(total, world, 1)[0]
        np.testing.assert_array_equal(np.load(str(out) + ".sub.npy"), ref["uk"][:, first:])


class _FakeCtl:
    """Stands in for ntm_mpc.NtmMpc: the N = 20 build by batch size (all-LDS up
    to 2048 scenarios, 8 per CU on 256 CUs) unless pinned."""

    def __init__(self):
        self.limit = -1

    def step_layout(self, B, cfg=None):
        lim = 2048 if self.limit < 0 else self.limit
        return "lds" if B <= lim else "far"

    def set_small_batch(self, n):
        self.limit = n


def test_pin_layout_follows_the_global_batch():
    """A far-build total sharded into all-LDS-size shards runs every shard on the
    far build (bitwise shard invariance needs one build)."""
    from ntm_mpc.dist import pin_layout, shard_range
    for total, world, want in ((100_000, 16, "far"), (16_384, 4, "far"), (4096, 4, "far"), (2048, 2, "lds"), (1024, 8, "lds")):
        ctl = _FakeCtl()
        assert pin_layout(ctl, total) == want
        for r in range(world):
            assert ctl.step_layout(shard_range(total, world, r)[1]) == want, (total, world, r)


def test_shard_range_partitions():
    from ntm_mpc.dist import shard_range
    for total in (0, 1, 7, 100000, 800000):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(c for _, c in spans) == total
            for (f0, c0), (f1, _) in zip(spans, spans[1:]):
                assert f0 + c0 == f1
