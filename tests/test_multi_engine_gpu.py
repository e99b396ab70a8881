"""The N > 1 path with real engines: two ranks on the one GPU, gloo
for the per-pair IQ broadcast (RCCL refuses two ranks on one device), each rank running its
shard of the chains on its own engine with block pairing (or quads) on (IqBroadcast(group=g)
makes every group of blocks contiguous on every rank).  The union of the ranks' chain outputs must be byte-identical to
one engine running every chain, and every rank must have paired its blocks (bench.py's N > 1
loop: the same calls in the same order)."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


FS, B, NB = 2400000, 1 << 17, 8
MODES = ["nfm", "usb", "am", "cw", "lsb", "nfm", "usb"]


def _stream(torch, hist):
    from openwebrx_amd import synth
    iq, offs = synth.make_iq(FS, NB * B, MODES)
    buf = torch.zeros(hist + iq.size, dtype=torch.complex64, device="cuda")
    buf[hist:] = torch.from_numpy(iq).to("cuda")
    return buf, offs


def _rank(rank, world, port, q, group):
    import torch  # before libowrx_amd.so (tests/conftest.py)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from openwebrx_amd import Engine, params
        from openwebrx_amd.multi import IqBroadcast, shard_chains
        eng = Engine(FS, max_block=B)
        eng.set_input_retention(8)
        eng.set_block_group(group)
        hist = eng.history
        t = torch.tensor([float(hist)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        hist_b = int(t.item())
        buf = offs = None
        if rank == 0:
            buf, offs = _stream(torch, hist_b)
        else:
            from openwebrx_amd import synth
            offs = synth.carrier_offsets(FS, len(MODES))
        items = list(enumerate(zip(offs, MODES)))
        mine = shard_chains(items, world, rank, key=lambda it: it[1][1])
        chains = [(i, eng.chain(params.chain_params(FS, o, m))) for i, (o, m) in mine]
        torch.cuda.synchronize()
        bc = IqBroadcast(torch, dist, "cuda", hist_b, B, stream=buf, retention=8, group=group)
        for j in range(NB):
            if j + 1 < NB:
                bc.issue(j + 1)
            tt, off = bc.wait(j)
            if rank != 0:
                eng.wait_stream(torch.cuda.current_stream().cuda_stream)
            eng.process_device(tt.data_ptr() + 8 * off, B)
        eng.sync()
        st = eng.stats()
        out = {i: (c.read_audio(), c.read_smeter().tobytes()) for i, c in chains}
        eng.close()
        dist.barrier()
        q.put((rank, {"blocks": st["blocks"], "out": out}))
        dist.destroy_process_group()
    except Exception as ex:  # reported to the parent, which fails the test
        q.put((rank, {"error": repr(ex)}))


@pytest.mark.parametrize("group", [2, 4])
def test_two_ranks_paired_equal_one_engine(group):
    import torch
    import torch.multiprocessing as mp
    from openwebrx_amd import Engine, params, synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q, group)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(30)
    for r in (0, 1):
        assert "error" not in res[r], res[r]
        # eight blocks as 8 / group engine blocks on both ranks: every group formed
        assert res[r]["blocks"] == NB // group, (r, res[r]["blocks"])
    got = {}
    for r in (0, 1):
        got.update(res[r]["out"])
    assert sorted(got) == list(range(len(MODES)))
    assert 0 < len(res[0]["out"]) < len(MODES)

    # one engine, every chain, the same blocks paired from one buffer
    eng = Engine(FS, max_block=B)
    eng.set_input_retention(8)
    eng.set_block_group(group)
    buf, offs = _stream(torch, eng.history)
    assert list(offs) == list(synth.carrier_offsets(FS, len(MODES)))
    chains = [eng.chain(params.chain_params(FS, o, m)) for o, m in zip(offs, MODES)]
    torch.cuda.synchronize()
    h = eng.history
    for j in range(NB):
        eng.process_device(buf.data_ptr() + 8 * (h + j * B), B)
    eng.sync()
    for i, c in enumerate(chains):
        audio, sm = c.read_audio(), c.read_smeter().tobytes()
        assert len(audio) > 0
        assert got[i][0] == audio, i
        assert got[i][1] == sm, i
    eng.close()
