"""N > 1 path on the CPU (gloo, world size 2): chain sharding and the per-block IQ broadcast
that bench.py / a multi-GPU server run over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from openwebrx_amd import params
from openwebrx_amd.multi import IqBroadcast, shard_chains


def test_shard_chains_balanced_and_disjoint():
    fs = 10000000
    items = [(o, m) for o, m in zip(range(0, 256 * 1000, 1000),
                                    (["nfm", "usb", "cw"] * 100)[:256])]
    key = lambda it: (params.decimation(fs, 12000)[0], it[1])  # (D, mode): same taps here
    for world in (1, 2, 4, 8):
        shards = [shard_chains(items, world, r, key) for r in range(world)]
        flat = [it for s in shards for it in s]
        assert sorted(flat) == sorted(items)
        sizes = [len(s) for s in shards]
        assert max(sizes) - min(sizes) <= 1
        for mode in ("nfm", "usb", "cw"):
            per = [sum(1 for it in s if it[1] == mode) for s in shards]
            assert max(per) - min(per) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, hist, block, nblocks, q, pipelined=False, retention=1,
            group=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(7)
    full = torch.complex(torch.randn(hist + nblocks * block, generator=g),
                         torch.randn(hist + nblocks * block, generator=g))
    bc = IqBroadcast(torch, dist, "cpu", hist, block, stream=full if rank == 0 else None,
                     retention=retention, group=group)
    ok = True
    live = []  # the windows an engine with this input retention may still read
    prev = None
    for i in range(nblocks):
        if pipelined and i + 1 < nblocks:
            bc.issue(i + 1)  # the next block's broadcast is in flight while block i is used
        t, off = bc.wait(i) if pipelined else bc.step(i)
        if group > 1 and i % group:
            # a group's later blocks sit right behind its first one in memory, so a grouping
            # engine (owrx_set_block_group) runs them as one engine block on every rank
            ok &= prev is not None and t.data_ptr() + 8 * off == prev[0].data_ptr() + 8 * (prev[1] + block)
        prev = (t, off)
        live = (live + [(i, t, off)])[-retention:]
        for k, tk, ok_off in live:  # none of them rewritten yet
            got = tk[ok_off - hist: ok_off + block]
            want = full[k * block: k * block + hist + block]
            ok &= bool(torch.equal(got, want))
    # every rank demodulates its own shard: no reduction, only a barrier for the timing
    dist.barrier()
    q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("pipelined,retention,group", [(False, 1, 1), (True, 1, 1), (True, 8, 1),
                                                        (False, 4, 2), (True, 4, 2), (True, 8, 2),
                                                        (True, 16, 4)])
def test_iq_broadcast_world2_gloo(pipelined, retention, group):
    """Every rank reconstructs [history | block] windows equal to rank 0's stream, with the
    broadcasts one at a time or pipelined one block ahead (bench.py's N > 1 loop); with input
    retention r (bench.py sets 8 at every N) the last r blocks' windows stay intact while the
    next broadcasts land.  group = 2 (4): blocks travel two (four) per broadcast into
    [history | group blocks] windows and each group is contiguous in memory on every rank, so
    ranks > 0 group blocks (owrx_set_block_group) as rank 0 does on its recording."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 64, 1000, 16, q, pipelined, retention, group))
             for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: True, 1: True}
