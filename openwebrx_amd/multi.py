"""Multi-GPU plumbing: one process per GPU, chains sharded across ranks, the
wideband IQ broadcast from rank 0 as the only exchange step.

* shard_chains -- round-robin within (decimation, taps, demodulator) groups, so every rank's
  DDC launch keeps the same per-group tile reuse and the ranks' loads differ by at most one
  chain per group.
* IqBroadcast -- rank 0 owns the stream (host ingest or an HBM-resident recording); each
  block goes to every rank with one torch.distributed broadcast (RCCL over xGMI with the
  "nccl" backend, gloo in the CPU tests).  Ranks > 0 assemble [history | block] windows (or
  [history | 2 blocks] with pair=True, so their engines pair blocks as rank 0's does), rotating
  enough of them for the engine's input retention (owrx_process_device contract,
  include/owrx_amd.h).
* Placement -- the same balance for the in-process drop-in (pycsdr shim, one engine per GPU
  in one OpenWebRX process), where chains come and go one at a time.
No reduction: every rank returns its own chains' outputs to the host.
"""
from collections import OrderedDict


def shard_chains(items, world, rank, key=lambda it: it):
    """This rank's share of `items`, dealt round-robin within groups of equal key(item);
    the dealer position carries over between groups so totals stay balanced."""
    groups = OrderedDict()
    for it in items:
        groups.setdefault(key(it), []).append(it)
    mine, pos = [], 0
    for members in groups.values():
        for it in members:
            if pos % world == rank:
                mine.append(it)
            pos += 1
    return mine


class Placement:
    """Online version of shard_chains for n engines: a new segment goes to the engine with
    the fewest segments of its group (same FirDecimate design, or the waterfalls), ties to the
    fewest segments overall, then the lowest index; release() when it leaves."""

    def __init__(self, n):
        self.n = n
        self.total = [0] * n
        self.groups = {}

    def place(self, key):
        g = self.groups.setdefault(key, [0] * self.n)
        slot = min(range(self.n), key=lambda k: (g[k], self.total[k], k))
        g[slot] += 1
        self.total[slot] += 1
        return slot

    def release(self, slot, key):
        self.groups[key][slot] -= 1
        self.total[slot] -= 1


class IqBroadcast:
    """Per-block IQ distribution.  step(i) returns (tensor, offset) such that the engine can
    process tensor[offset : offset + block] with tensor[offset - history : offset] holding
    the preceding samples.

    Pipelined use (issue / wait): issue(i + 1) is enqueued before block i is processed, so the
    broadcast of the next block overlaps this block's host and GPU work.  Ranks > 0 therefore
    rotate retention + 2 windows (three at retention 1): issue(i + 1) rewrites block
    i + 1 - nwin's window, which the engine has finished once owrx_process_device(i) returned
    (owrx_set_input_retention's contract: blocks before k - retention + 1 are released).

    pair=True (ranks that run owrx_set_block_pairing, round 6): blocks 2u and 2u + 1 travel in
    one broadcast into one window [history | block 2u | block 2u + 1], so on every rank the two
    blocks of a pair are contiguous in memory and the engine runs them as one engine block,
    exactly as rank 0 does on its resident recording.  A window then covers two blocks and the
    ring holds retention // 2 + 3 of them.  group=g: g blocks per broadcast and window (the
    engines' owrx_set_block_group), retention // g + 3 windows."""

    NWIN = 3

    def __init__(self, torch, dist, device, history, block, src=0, stream=None, retention=1,
                 pair=False, group=None):
        self.torch, self.dist = torch, dist
        self.history, self.block, self.src = history, block, src
        self.rank = dist.get_rank()
        self.stream = stream  # rank src: complex64 tensor [history | blocks...]
        # blocks per broadcast (and per window): the engines' block group (owrx_set_block_group;
        # pair=True: 2)
        self.per = max(1, int(group)) if group is not None else (2 if pair else 1)
        self.pending = {}     # unit -> async broadcast handle
        self.next_issue = 0   # broadcasts are enqueued in unit order on every rank
        # an engine with input retention r still reads blocks k - r + 1 .. k after
        # owrx_process_device(k) returned, and block k + 1's broadcast is issued before block k is
        # processed: the units of blocks k - r .. k + 1 stay intact, r + 2 windows unpaired (3 for
        # r = 1), r // 2 + 3 paired
        if self.per > 1:
            self.nwin = max(self.NWIN, int(retention) // self.per + 3)
        else:
            self.nwin = max(self.NWIN, int(retention) + 2)
        if self.rank != src:
            self.windows = [torch.zeros(history + self.per * block, dtype=torch.complex64,
                                        device=device) for _ in range(self.nwin)]

    def _view(self, u):
        """Broadcast unit u: (the part that travels, the tensor holding it, offset of its first
        block)."""
        h, b = self.history, self.per * self.block
        lo = 0 if u == 0 else h  # the first broadcast also carries the initial history
        if self.rank == self.src:
            return self.stream[lo + u * b if u else 0: h + (u + 1) * b], self.stream, h + u * b
        w = self.windows[u % self.nwin]
        return w[lo:h + b], w, h

    def issue(self, i):
        """Enqueue the broadcasts up to block i's (not waiting for them), in block order: the
        ranks' collectives must match one for one."""
        u = i // self.per
        while self.next_issue <= u:
            self._issue(self.next_issue)
            self.next_issue += 1

    def _issue(self, u):
        h, b = self.history, self.per * self.block
        if self.rank != self.src and u > 0:
            # the window starts with the previous unit's last `history` samples: that unit's
            # broadcast must land first (a stream-level wait with RCCL)
            prev = self.pending.get(u - 1)
            if prev is not None:
                prev.wait()
            w, pw = self.windows[u % self.nwin], self.windows[(u - 1) % self.nwin]
            w[:h].copy_(pw[b:b + h])
        part, _, _ = self._view(u)
        self.pending[u] = self.dist.broadcast(self.torch.view_as_real(part), src=self.src,
                                              async_op=True)

    def wait(self, i):
        """Block i's (tensor, offset) once its broadcast has landed (issued if it was not)."""
        self.issue(i)
        u = i // self.per
        w = self.pending.pop(u, None)
        if w is not None:
            w.wait()
        # older handles whose windows issue(i) already waited for
        for k in [k for k in self.pending if k < u]:
            self.pending.pop(k)
        _, t, off = self._view(u)
        return t, off + (i % self.per) * self.block

    def step(self, i):
        """Unpipelined: broadcast block i and return it."""
        return self.wait(i)
