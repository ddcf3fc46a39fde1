"""Long units on the side stream: encode_tiled_kernel and the decode
fallback take the long units from a device queue on a side stream of the caller's
stream, joined back into it. These tests check that the fork/join orders them with
the caller's own work:
- on a caller-created (non-default) stream, with the result read right after a
  synchronisation of that stream only;
- back-to-back batches of different long-unit mixes, so a later batch's queue reset
  cannot overtake an earlier batch's workers;
- captured into a hipGraph (torch.cuda.graph) and replayed on new data, also after a
  larger eager batch on the capturing stream (the queue grows; the captured one must
  stay valid), and with a caller workspace while an eager batch runs on another
  stream;
- a batch with no long units and one of long units only (the empty-queue and
  all-queue ends).
Every unit is checked against the oracle (message.zig:200-271 / 88-145) or by
decode(encode(x)) == x.
"""
import numpy as np
import pytest

import capnp_packed as cp
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


DEV = "cuda"


def mixed_sizes(n, seed, long_every=7, huge_every=61):
    rng = np.random.default_rng(seed)
    sizes = (rng.integers(1, 512, n) * 8).astype(np.int64)            # one tile
    sizes[::long_every] = rng.integers(513, 8192, len(sizes[::long_every])) * 8  # tiled / fallback
    sizes[::huge_every] = rng.integers(8193, 24576, len(sizes[::huge_every])) * 8  # > 64 KiB: front of the queue
    return sizes


class Batch:
    def __init__(self, sizes, seed, thr=128):
        n = len(sizes)
        self.n = n
        self.sizes = torch.from_numpy(sizes).to(DEV)
        self.in_off = torch.zeros(n, dtype=torch.int64, device=DEV)
        self.in_off[1:] = torch.cumsum(self.sizes, 0)[:-1]
        self.U = int(sizes.sum())
        self.seed, self.thr = seed, thr
        self.d_in = cp.generate(1, self.U, seed=seed, zero_thresh=thr, device=DEV)
        self.cap = (self.sizes // 8) * 10
        slots = (self.cap + 15) // 16 * 16
        self.pk_off = torch.zeros(n, dtype=torch.int64, device=DEV)
        self.pk_off[1:] = torch.cumsum(slots, 0)[:-1]
        self.d_pk = torch.zeros(int(slots.sum().item()), dtype=torch.uint8, device=DEV)
        self.plen = torch.zeros(n, dtype=torch.int64, device=DEV)
        self.pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
        self.d_out = torch.zeros(self.U, dtype=torch.uint8, device=DEV)
        self.ulen = torch.zeros(n, dtype=torch.int64, device=DEV)
        self.ust = torch.full((n,), -1, dtype=torch.int32, device=DEV)

    def run(self, stream=None, ws=None):
        cp.encode_batch(self.d_in, self.in_off, self.sizes, self.d_pk, self.pk_off, self.cap, self.plen, self.pst,
                        stream=stream, ws=ws)
        cp.decode_batch(self.d_pk, self.pk_off, self.plen, self.d_out, self.in_off, self.sizes, self.ulen, self.ust,
                        stream=stream, ws=ws)

    def reset(self, seed):
        cp.generate(1, self.U, seed=seed, zero_thresh=self.thr, out=self.d_in, device=DEV)
        self.pst.fill_(-1)
        self.ust.fill_(-1)
        self.d_out.zero_()

    def check_roundtrip(self):
        assert (self.pst == 0).all().item() and (self.ust == 0).all().item()
        assert torch.equal(self.ulen, self.sizes)
        assert torch.equal(self.d_out, self.d_in)

    def check_oracle(self, units):
        h_in = self.d_in.cpu().numpy()
        pk = self.d_pk.cpu().numpy()
        plen, off, pko = self.plen.cpu().numpy(), self.in_off.cpu().numpy(), self.pk_off.cpu().numpy()
        sz = self.sizes.cpu().numpy()
        for i in units:
            st, exp = oracle.pack(h_in[off[i]:off[i] + sz[i]].tobytes())
            assert st == oracle.OK and int(plen[i]) == len(exp), f"unit {i} ({sz[i]} B): packed length"
            assert pk[pko[i]:pko[i] + len(exp)].tobytes() == exp, f"unit {i} ({sz[i]} B): packed bytes"


def test_side_stream_on_caller_stream():
    b = Batch(mixed_sizes(3000, 1), seed=0xC0DE0101)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        b.run(stream=s)
    s.synchronize()  # only the caller's stream: the join must cover the side work
    b.check_roundtrip()
    long_units = [i for i, x in enumerate(b.sizes.cpu().numpy()) if x > 4096]
    b.check_oracle(long_units[:200] + list(range(0, 3000, 97)))


@pytest.mark.parametrize("thr", [26, 128, 230])
def test_back_to_back_batches(thr, decoder):
    # three batches, launched without synchronisation in between: each batch resets the
    # shared queue on the side stream after the previous batch's workers
    bs = [Batch(mixed_sizes(n, 10 + k, long_every=le), seed=0xC0DE0200 + k, thr=thr)
          for k, (n, le) in enumerate([(2000, 5), (700, 2), (4000, 1000)])]
    for b in bs:
        b.run()
    torch.cuda.synchronize()
    for b in bs:
        b.check_roundtrip()
    bs[1].check_oracle(range(0, 700, 3))


def test_no_long_units_and_only_long_units():
    short = Batch(np.full(5000, 4096, dtype=np.int64), seed=0xC0DE0301)
    only = Batch((np.arange(1, 65) * 4104).astype(np.int64), seed=0xC0DE0302)
    short.run()
    only.run()
    torch.cuda.synchronize()
    short.check_roundtrip()
    only.check_roundtrip()
    only.check_oracle(range(64))


def test_graph_capture_replay(decoder):
    b = Batch(mixed_sizes(1500, 3), seed=0xC0DE0401)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        b.run(stream=s)  # warm-up: sizes this stream's queue before capture
    s.synchronize()
    b.check_roundtrip()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        b.run()
    # new data in the same buffers, then replay the captured encode + decode
    b.reset(0xC0DE0402)
    g.replay()
    torch.cuda.synchronize()
    b.check_roundtrip()
    long_units = [i for i, x in enumerate(b.sizes.cpu().numpy()) if x > 4096]
    b.check_oracle(long_units[:100])


def test_graph_replay_after_larger_eager_batch():
    # the capturing stream's queue grows for a larger eager batch after the capture:
    # the old queue, baked into the graph, must stay allocated
    small = Batch(mixed_sizes(600, 4), seed=0xC0DE0411)
    big = Batch(mixed_sizes(5000, 5), seed=0xC0DE0412)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        small.run(stream=s)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        small.run()
    with torch.cuda.stream(s):
        big.run(stream=s)  # grows s's queue
    s.synchronize()
    big.check_roundtrip()
    small.reset(0xC0DE0413)
    torch.cuda.empty_cache()
    g.replay()
    torch.cuda.synchronize()
    small.check_roundtrip()
    long_units = [i for i, x in enumerate(small.sizes.cpu().numpy()) if x > 4096]
    small.check_oracle(long_units[:60])


def test_graph_with_workspace_beside_eager_stream():
    # a graph captured with its own workspace replays while an eager batch runs on
    # another stream: nothing of either is shared
    a = Batch(mixed_sizes(1200, 6), seed=0xC0DE0421)
    e = Batch(mixed_sizes(2500, 7), seed=0xC0DE0422)
    ws = cp.workspace(a.n, device=DEV)
    s, t = torch.cuda.Stream(), torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    t.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        a.run(ws=ws)  # no warm-up needed: the workspace is the queue
    a.reset(0xC0DE0423)
    with torch.cuda.stream(s):
        g.replay()
    with torch.cuda.stream(t):
        e.run(stream=t)
    torch.cuda.synchronize()
    a.check_roundtrip()
    e.check_roundtrip()
    e.check_oracle([i for i, x in enumerate(e.sizes.cpu().numpy()) if x > 4096][:60])


def test_workspace_too_small_is_rejected():
    b = Batch(mixed_sizes(100, 8), seed=0xC0DE0431)
    ws = cp.workspace(10, device=DEV)
    with pytest.raises(cp.InvalidArgument):
        b.run(ws=ws)


def test_misaligned_workspace_is_rejected():
    b = Batch(mixed_sizes(100, 8), seed=0xC0DE0432)
    ws = cp.workspace(b.n + 64, device=DEV)
    with pytest.raises(cp.InvalidArgument):
        b.run(ws=ws[16:])  # 128 B past the 256-B aligned base
    b.run(ws=ws)
    torch.cuda.synchronize()
    b.check_roundtrip()


def test_queue_growth_is_bounded_and_released():
    """Growing batches on one stream: the library's queue grows geometrically, replaced
    queues are freed (none was captured), device memory stays bounded, and
    capnp_packed_stream_release drops the context."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    wb = cp.lib().capnp_packed_batch_workspace_bytes
    sizes_all = mixed_sizes(4200, 9, long_every=50, huge_every=997)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    grows, last = 0, 0
    with torch.cuda.stream(s):
        for n in range(200, 4200, 97):
            b = Batch(sizes_all[:n], seed=0xC0DE0440 + n)
            b.run(stream=s)
            qb, kept = cp.stream_queue_info(s)
            assert kept == 0 and wb(n) <= qb <= wb(2 * n + 1)
            grows += qb != last
            last = qb
    s.synchronize()
    b.check_roundtrip()
    assert grows <= 6  # 200 -> 4200 units at >= 2x per growth: at most 5 growths after the first
    del b
    torch.cuda.empty_cache()
    free1 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 <= wb(2 * 4200) + (64 << 20), (free0, free1)
    cp.stream_release(s)
    assert cp.stream_queue_info(s) == (0, 0)
    # the stream works again after a release (a new context)
    b = Batch(mixed_sizes(300, 10), seed=0xC0DE0450)
    with torch.cuda.stream(s):
        b.run(stream=s)
    s.synchronize()
    b.check_roundtrip()
    cp.stream_release(s)


def test_captured_queue_is_kept_until_release():
    small = Batch(mixed_sizes(600, 11), seed=0xC0DE0461)
    big = Batch(mixed_sizes(5000, 12), seed=0xC0DE0462)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        small.run(stream=s)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        small.run()
    with torch.cuda.stream(s):
        big.run(stream=s)  # grows: the captured queue is kept
    s.synchronize()
    assert cp.stream_queue_info(s)[1] == 1
    small.reset(0xC0DE0463)
    g.replay()
    torch.cuda.synchronize()
    small.check_roundtrip()
    big.check_roundtrip()
    del g
    cp.stream_release(s)
    assert cp.stream_queue_info(s) == (0, 0)


def test_tile_table_overflow_goes_serial():
    # Long-unit encode is tile-parallel through a tile table of n + 65536 tiles
    # (long_tiles_kernel). Three units of 30000 tiles (123 MB each) need 90000 > 65539:
    # the unit whose reservation does not fit is encoded by the serial tiled kernel
    # instead. Both paths must give the oracle's bytes.
    words = 30000 * 512
    b = Batch(np.array([words * 8, 4096 * 3 + 8, words * 8, words * 8], dtype=np.int64), seed=0xC0DE0601)
    b.run()
    torch.cuda.synchronize()
    b.check_roundtrip()
    b.check_oracle(range(4))
    # the encoded-size pass over the same tiles
    plen2 = torch.zeros_like(b.plen)
    st2 = torch.full_like(b.pst, -1)
    cp.encoded_size_batch(b.d_in, b.in_off, b.sizes, plen2, st2)
    torch.cuda.synchronize()
    assert (st2 == 0).all().item() and torch.equal(plen2, b.plen)


def test_few_large_units():
    # a batch of a few large units gets up to a wave per unit (round 1 sized the
    # long-unit grids by unit count / 256: a handful of waves for the whole batch)
    b = Batch(np.full(8, 262144, dtype=np.int64), seed=0xC0DE0701)
    b.run()
    torch.cuda.synchronize()
    b.check_roundtrip()
    b.check_oracle(range(8))
