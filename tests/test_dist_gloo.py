"""world_size 2, 3 and 4 gloo tests of the sharded loop-ICP exchange (CPU).

Each rank owns a contiguous range of 4096-point records (lio_icp_shard_range),
all-gathers its record statistics through lio_gpu.dist (the same code path the
ctypes callback uses on the GPU box, there over RCCL) and combines them in
record order (lio_icp_combine, C++).  Every rank must get the bit-identical
17 statistics that a single rank gets — which is what makes the sharded ICP
transform identical for 1/2/4/8 GPUs.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

NS = 300_001


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _records(ns):
    rng = np.random.default_rng(1234)
    nrec = (ns + 4095) // 4096
    return rng.normal(size=(nrec, 20)) * 1e3


def _worker(rank, world, port, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "fast-lio-sam_gps_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ctypes as C

        from lio_gpu import dist as ld

        recs = _records(NS)
        b, n = ld.shard_range(NS, rank, world)
        r0 = b // 4096
        mine = recs[r0: r0 + (n + 4095) // 4096]
        nrec = len(recs)
        slot = -(-nrec // world)
        send = np.zeros((slot, 20))
        send[: len(mine)] = mine
        # drive the exchange through the ctypes callback exactly as liblio_gpu does
        cb = ld.make_allgather()
        recv = np.zeros(slot * 20 * world)
        rc = cb(send.ravel().ctypes.data_as(C.POINTER(C.c_double)), send.size,
                recv.ctypes.data_as(C.POINTER(C.c_double)), None)
        assert rc == 0
        out = ld.combine(recv, NS, world)
        q.put((rank, out.tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_icp_exchange_gloo(world):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fast-lio-sam_gps_amd"))
    from lio_gpu import dist as ld

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    got = [q.get(timeout=120) for _ in range(world)]
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    recs = _records(NS)
    ref = ld.combine(recs.ravel(), NS, 1)
    for rank, b in got:
        np.testing.assert_array_equal(np.frombuffer(b), ref)


def _shm_worker(rank, world, name, rounds, q):
    """Rank of the C++ shared-memory all-gather (lio_shm_exchange_*, the transport of lio_icp_set_shard_shm):
    rank 0 opens first (ordered here by a queue handshake), then `rounds` exchanges of record sets with no
    Python callback inside the library; every rank's combine of every round must equal one rank's."""
    import sys
    import time

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "fast-lio-sam_gps_amd"))
    from lio_gpu import dist as ld

    if rank != 0:
        time.sleep(0.3)  # rank 0 creates the segment first (the library retries the open for 5 s anyway)
    recs = _records(NS)
    nrec = len(recs)
    slot = -(-nrec // world)
    b, n = ld.shard_range(NS, rank, world)
    r0 = b // 4096
    ex = ld.ShmExchange(name, rank, world, slot * 20)
    outs = []
    for k in range(rounds):
        mine = recs[r0: r0 + (n + 4095) // 4096] * (k + 1)  # different data every round (buffer reuse)
        send = np.zeros((slot, 20))
        send[: len(mine)] = mine
        recv = ex.allgather(send.ravel())
        outs.append(ld.combine(recv, NS, world).tobytes())
    ex.close()
    q.put((rank, outs))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_shm_exchange_cpp(world):
    """The C++ shared-memory exchange the one-node multi-rank loop ICP uses (no Python in
    the per-pass exchange): 50 rounds, alternating buffer sets, one barrier per round; every rank's record-order
    combine equals the single-rank combine of the same records, round by round."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fast-lio-sam_gps_amd"))
    from lio_gpu import dist as ld

    rounds = 50
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/lio_test_{os.getpid()}_{world}"
    procs = [ctx.Process(target=_shm_worker, args=(r, world, name, rounds, q)) for r in range(world)]
    [p.start() for p in procs]
    got = [q.get(timeout=120) for _ in range(world)]
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    recs = _records(NS)
    for rank, outs in got:
        assert len(outs) == rounds
        for k, b in enumerate(outs):
            np.testing.assert_array_equal(np.frombuffer(b), ld.combine((recs * (k + 1)).ravel(), NS, 1))


def _windows(world):
    """Synthetic windows of a chain split over `world` ranks (rank 1 empty when world > 2): per rank its elements
    of 6 chains and its event lists (local positions, local increment prefixes, values)."""
    rng = np.random.default_rng(7)
    sizes = [int(v) for v in rng.integers(2000, 9000, world)]
    if world > 2:
        sizes[1] = 0
    out = []
    for r, n in enumerate(sizes):
        x = (rng.normal(3.0, 40.0, (6, n))).astype(np.float32)
        evs = []
        for c in range(6):
            ne = int(rng.integers(0, 60)) if n else 0
            pos = np.sort(rng.choice(n, ne, replace=False)).astype(np.int64) if ne else np.zeros(0, np.int64)
            P = np.sort(rng.integers(0, 1 << 40, ne)).astype(np.uint64)
            evs.append((pos, P, x[c, pos] if ne else np.zeros(0, np.float32), int(rng.integers(1 << 40, 1 << 41))))
        out.append((n, x, evs))
    return out


def _shard_msg_worker(rank, world, port, slot, q):
    """One rank of the sharded float chains' exchange on CPU: its totals and its event
    message in the documented layout (lio_gpu.dist.SEQ_*), all-gathered through the ctypes callback the library
    calls (gloo), then the host mirrors of seq_shard_offsets / seq_shard_merge (the device kernels' own code)."""
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "fast-lio-sam_gps_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ctypes as C

        from lio_gpu import dist as ld

        n, x, evs = _windows(world)[rank]
        cb = ld.make_allgather()
        # block sums: [0] n, per chain nb_slot (block double sum, block sum |x|)
        nbs = 10
        tw = ld.SEQ_TOT_HDR + 6 * 2 * nbs
        tot = np.zeros(tw)
        tot[0] = n
        for c in range(6):
            for j, b0 in enumerate(range(0, n, ld.SEQ_BLOCK)):
                blk = x[c, b0:b0 + ld.SEQ_BLOCK].astype(np.float64)
                tot[ld.SEQ_TOT_HDR + c * 2 * nbs + 2 * j] = float(np.sum(blk))
                tot[ld.SEQ_TOT_HDR + c * 2 * nbs + 2 * j + 1] = float(np.sum(np.abs(blk)))
        rtot = np.zeros(tw * world)
        assert cb(tot.ctypes.data_as(C.POINTER(C.c_double)), tw, rtot.ctypes.data_as(C.POINTER(C.c_double)), None) == 0
        off = ld.seq_shard_offsets(rtot, tw, nbs, rank, world, 6)
        # events
        words = ld.SEQ_HDR_WORDS + 6 * 2 * slot
        msg = np.zeros(words)
        mi = msg.view(np.int64)
        mi[0] = n
        for c, (pos, P, xv, ptot) in enumerate(evs):
            mi[2 + c] = np.int64(np.uint64(ptot).view(np.int64))
            mi[2 + ld.SEQ_MAX_CHAINS + c] = len(pos)
            msg[2 + 2 * ld.SEQ_MAX_CHAINS + c] = float(x[c, 0]) if n else 0.0
            m = min(len(pos), slot)
            b = ld.SEQ_HDR_WORDS + c * 2 * slot
            mi[b:b + 2 * m:2] = P[:m].view(np.int64)
            mi[b + 1:b + 2 * m:2] = (pos[:m].astype(np.uint64) | (xv[:m].view(np.uint32).astype(np.uint64) << np.uint64(32))).view(np.int64)
        rmsg = np.zeros(words * world)
        assert cb(msg.ctypes.data_as(C.POINTER(C.c_double)), words, rmsg.ctypes.data_as(C.POINTER(C.c_double)), None) == 0
        merged = [ld.seq_shard_merge(rmsg, words, world, slot, c, 4096) for c in range(6)]
        q.put((rank, off, merged))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,slot", [(2, 64), (3, 64), (4, 64), (3, 16)])
def test_sharded_float_chain_messages_gloo(world, slot):
    """The sharded PCL float statistics' messages over gloo: every rank gets the same common
    floors and totals, its window's starting prefix is the double sum of the windows before it, and the merged
    event lists are every rank's events in element order (positions and increment prefixes moved by the ranks
    before); a list longer than the slot is flagged (bit 2) on every rank, so every rank takes the same re-exchange."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fast-lio-sam_gps_amd"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_msg_worker, args=(r, world, port, slot, q)) for r in range(world)]
    [p.start() for p in procs]
    got = sorted((q.get(timeout=120) for _ in range(world)), key=lambda t: t[0])
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    win = _windows(world)
    sizes = [w[0] for w in win]
    for rank, off, merged in got:
        off0, var0, fl, gbase, ng = off
        assert gbase == sum(sizes[:rank]) and ng == sum(sizes)
        for c in range(6):  # the prefix: the blocks of the windows before, block sums added in chain order
            want = 0.0
            for r in range(rank):
                for b0 in range(0, sizes[r], 1024):
                    want = want + float(np.sum(win[r][1][c, b0:b0 + 1024].astype(np.float64)))
            assert off0[c] == want
        np.testing.assert_array_equal(fl, got[0][1][2])  # the floors: identical on every rank
        np.testing.assert_array_equal(var0 >= 0, True)
        for c in range(6):
            m = merged[c]
            lens = [len(w[2][c][0]) for w in win]
            if max(lens) > slot:
                assert m["bad"] & 2 and m["longest"] == max(lens)
                continue
            assert m["bad"] == 0 and m["nev"] == sum(lens)
            base = np.cumsum([0] + sizes[:-1])
            pb = np.cumsum([0] + [w[2][c][3] for w in win[:-1]]).astype(np.uint64)
            pos = np.concatenate([w[2][c][0] + base[r] for r, w in enumerate(win)])
            P = np.concatenate([w[2][c][1] + pb[r] for r, w in enumerate(win)])
            xs = np.concatenate([w[2][c][2] for w in win])
            np.testing.assert_array_equal(m["pos"], pos)
            np.testing.assert_array_equal(m["P"], P)
            np.testing.assert_array_equal(m["x"], xs)
            assert m["ptot"] == int(sum(w[2][c][3] for w in win)) % (1 << 64)
            first = next(r for r in range(world) if sizes[r])
            assert m["x0"] == float(win[first][1][c][0])


def test_shm_exchange_reopen_same_name():
    """a second segment under the same name (a handle re-sharded, or two handles sharing a name)
    must survive the first one's close — the name is unlinked once every rank has attached, and a close only
    unlinks a name that still refers to its own segment."""
    import sys
    import threading

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fast-lio-sam_gps_amd"))
    from lio_gpu import dist as ld

    name = f"/lio_reopen_{os.getpid()}"
    a0 = ld.ShmExchange(name, 0, 2, 8)
    a1 = ld.ShmExchange(name, 1, 2, 8)
    b0 = ld.ShmExchange(name, 0, 2, 8)  # same name again (rank 0 first, as the callers order it)
    a0.close()  # must not remove b0's segment
    a1.close()
    b1 = ld.ShmExchange(name, 1, 2, 8)  # opens b0's segment (failed with the old close)
    out = [None, None]

    def run(ex, r):
        out[r] = ex.allgather(np.full(8, float(r + 1)))

    th = [threading.Thread(target=run, args=(ex, r)) for r, ex in enumerate((b0, b1))]
    [t.start() for t in th]
    [t.join(timeout=30) for t in th]
    for r in range(2):
        np.testing.assert_array_equal(out[r], np.concatenate([np.full(8, 1.0), np.full(8, 2.0)]))
    b0.close()
    b1.close()
    assert not os.path.exists(f"/dev/shm{name}")


def test_shm_exchange_timeout_poisons_segment():
    """a barrier that times out leaves its arrival counted, so the segment is poisoned — every later
    all-gather on it fails on every rank instead of releasing early with stale records."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fast-lio-sam_gps_amd"))
    from lio_gpu import _capi, dist as ld

    name = f"/lio_poison_{os.getpid()}"
    e0 = ld.ShmExchange(name, 0, 2, 4, timeout_s=0.2)
    e1 = ld.ShmExchange(name, 1, 2, 4, timeout_s=0.2)
    with pytest.raises(_capi.LioError, match="did not arrive"):
        e0.allgather(np.ones(4))  # rank 1 never arrives
    for ex in (e1, e0):
        with pytest.raises(_capi.LioError, match="poisoned"):
            ex.allgather(np.ones(4))
    e0.close()
    e1.close()
    with pytest.raises(_capi.LioError, match="another world size"):  # checked on open by ranks other than 0
        f0 = ld.ShmExchange(name, 0, 3, 4)
        try:
            ld.ShmExchange(name, 1, 2, 4)
        finally:
            f0.close()
