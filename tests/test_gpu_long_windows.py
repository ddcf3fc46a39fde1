"""Long units, window-parallel decode (message.zig:88-145).

Packed units too long for the indexed decoder are cut into 4,608-B windows at fixed
positions; a spec pass resolves each window's chain for every entry in its first 64
bytes, a resolve pass chains the windows of a unit (and re-stages the windows whose entry
the spec pass could not resolve), and a fill pass expands each window. These tests aim at
each of those cases and compare every unit with the oracle (status, length, bytes):
- random long units at p = 0.1 / 0.5 / 0.9 (5 KB .. 1.5 MB packed), unaligned bases;
- records that straddle a window boundary at every entry depth that matters: 0 .. 9
  (mixed records), 15 .. 17 and 63 .. 65 (the spec pass's entry range), 100 .. 2000 (an
  FF record landing deep: the resolve pass re-stages the window);
- zero-run streams ("00 FF" records: 256 words per 2 bytes; the largest word deltas);
- truncated units (UnexpectedEof in the first, a middle and the last window, inside an
  FF run) and slots one word too small (OutOfSpace): the slot is left untouched, as the
  reference returns no output for these (message.zig:90);
- more windows than the window table holds (n / 8 + 32768): those units take the serial
  windowed decoder, the others the table.
"""
import numpy as np
import pytest

import capnp_packed as cp
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"
WIN = 4608
CANARY = 0xA5


def decode_units(units, caps=None, base_pad=None, seed=0):
    """Decode host packed units (bytes) as one batch from a dense, unaligned packed buffer
    into canary-filled slots; returns (status, out_len, outputs, slots_untouched)."""
    rng = np.random.default_rng(seed)
    n = len(units)
    pads = base_pad if base_pad is not None else rng.integers(0, 16, n)
    offs, pos = [], 0
    for u, p in zip(units, pads):
        pos += int(p)
        offs.append(pos)
        pos += len(u)
    buf = np.zeros(pos + 16, dtype=np.uint8)
    for u, o in zip(units, offs):
        buf[o:o + len(u)] = np.frombuffer(u, dtype=np.uint8)
    exp = [oracle.unpack(u) for u in units]
    if caps is None:
        caps = [max(8, len(e[1])) for e in exp]
    slot_off, q = [], 0
    for c in caps:
        slot_off.append(q)
        q += (int(c) + 16 + 7) // 8 * 8
    d_in = torch.from_numpy(buf).to(DEV)
    d_out = torch.full((q + 16,), CANARY, dtype=torch.uint8, device=DEV)
    t = lambda a: torch.tensor(a, dtype=torch.int64, device=DEV)
    out_len = torch.zeros(n, dtype=torch.int64, device=DEV)
    st = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_in, t(offs), t([len(u) for u in units]), d_out, t(slot_off), t(caps), out_len, st)
    torch.cuda.synchronize()
    h = d_out.cpu().numpy()
    st, out_len = st.cpu().numpy(), out_len.cpu().numpy()
    outs, untouched = [], []
    for i in range(n):
        L = int(out_len[i]) if st[i] == oracle.OK else 0
        outs.append(h[slot_off[i]:slot_off[i] + L].tobytes())
        rest = h[slot_off[i] + L:slot_off[i] + int(caps[i]) + 16]
        untouched.append(bool((rest == CANARY).all()))
    return st, out_len, outs, untouched, exp


def check(units, caps=None, seed=0):
    st, out_len, outs, untouched, exp = decode_units(units, caps, seed=seed)
    for i, (es, eb) in enumerate(exp):
        cap = len(eb) if caps is None else caps[i]
        if es == oracle.OK and len(eb) > cap:
            es = cp.OUT_OF_SPACE
        assert st[i] == es, f"unit {i} ({len(units[i])} B packed): status {st[i]} != {es}"
        if es == oracle.OK:
            assert int(out_len[i]) == len(eb), f"unit {i}: length"
            assert outs[i] == eb, f"unit {i}: bytes"
        elif es == cp.OUT_OF_SPACE:
            assert int(out_len[i]) == len(eb), f"unit {i}: required length"
        assert untouched[i], f"unit {i}: bytes written past the output (or into a failed unit's slot)"


def random_units(rng, n, thr, lo_words, hi_words):
    sizes = rng.integers(lo_words, hi_words, n) * 8
    data = oracle.generate(1, int(sizes.sum()), seed=int(rng.integers(1 << 30)), zero_thresh=thr)
    units, o = [], 0
    for s in sizes:
        st, p = oracle.pack(data[o:o + s].tobytes())
        assert st == oracle.OK
        units.append(p)
        o += s
    return units


@pytest.mark.parametrize("thr", [26, 128, 230])
def test_random_long_units(thr):
    rng = np.random.default_rng(thr)
    units = random_units(rng, 40, thr, 800, 20000)                 # 6 KB .. 160 KB unpacked
    units += random_units(rng, 3, thr, 150000, 190000)             # ~1.2-1.5 MB
    units = [u for u in units if len(u) > 5120] + [units[0][:0] + b"\x00\x00"]  # plus one short unit
    check(units, seed=thr)


def filler(n):
    """n >= 2 packed bytes of 2- and 3-byte mixed records (tag 0x01 + 1 byte, tag 0x03 + 2 bytes)."""
    assert n >= 2
    twos = {0: 0, 1: 2, 2: 1}[n % 3]
    return b"\x01\x07" * twos + b"\x03\x05\x09" * ((n - 2 * twos) // 3)


def ff_record(c, fill=0x11):
    return b"\xff" + bytes([fill] * 8) + bytes([c]) + bytes([(fill + 1 + i) % 255 + 1 for i in range(8 * c)])


@pytest.mark.parametrize("depths", [list(range(0, 10)), [15, 16, 17, 31, 32, 33], [63, 64, 65, 72, 73, 100],
                                    [145, 146, 147, 500, 1000, 2040]])
def test_records_straddling_window_boundaries(depths):
    units = []
    for d in depths:
        # a record that starts before X_1 = 4608 and ends d bytes past it: a mixed record
        # (<= 8 B) for d <= 7, else an FF record of 10 + 8c > d bytes
        if d >= 8:
            c = min(255, max(0, (d - 2) // 8))
            rec = ff_record(c)
        else:
            rec = b"\x7f" + bytes(range(1, 8))   # 8-byte record (tag + 7 bytes)
        s = WIN + d - len(rec)
        assert 0 < s < WIN
        body = filler(s) + rec
        # and the same depth at X_2 = 9216
        s2 = 2 * WIN + d - len(rec) - len(body)
        body += filler(s2) + rec + filler(1500)
        units.append(body)
        units.append(body[:len(body) - 700])     # the same unit cut inside a record (EOF) ...
        units.append(body[:len(body) - 699])     # ... and at a record boundary
    check(units, seed=len(depths))


def test_zero_runs_and_literal_runs():
    units = [
        b"\x00\xff" * 6000,                                        # 12 KB -> 12 MB of zeros
        (b"\x00\xff" * 70 + filler(300)) * 40,                     # zero runs inside lanes 0/1
        ff_record(255) * 12,                                       # 2 KB literal runs
        (ff_record(255) + b"\x00\x00" + filler(9)) * 9,
        (b"\x00\x03" + ff_record(3) + b"\x0f\x01\x02\x03\x04") * 800,
    ]
    check(units)


def test_truncated_units_write_nothing():
    rng = np.random.default_rng(7)
    base = random_units(rng, 6, 26, 3000, 6000)                   # p = 0.1: many FF runs
    units = []
    for u in base:
        for cut in (1, 17, 4000, WIN + 3, len(u) // 2, len(u) - 1):
            if 5120 < len(u) - cut:
                units.append(u[:len(u) - cut])
    units.append(ff_record(255) * 3 + b"\xff" + bytes(8) + b"\x10" + bytes(40))  # FF run cut short
    units.append(b"\x00\xff" * 3000 + b"\x00")                    # count byte missing
    exp = [oracle.unpack(u)[0] for u in units]
    assert cp.UNEXPECTED_EOF in exp and oracle.OK in exp
    check(units, seed=7)


def test_out_of_space_writes_nothing():
    rng = np.random.default_rng(8)
    units = random_units(rng, 12, 128, 1000, 9000)
    units = [u for u in units if len(u) > 5120]
    sizes = [len(oracle.unpack(u)[1]) for u in units]
    caps = [s - 8 if i % 2 else s for i, s in enumerate(sizes)]
    check(units, caps=caps, seed=8)


def test_more_windows_than_the_table_holds():
    # 6 units of ~46 MB packed (p = 0.1): ~60,000 windows > 6 / 8 + 32768; the units that
    # do not fit go to the serial decoder. Checked by a device round trip.
    n, ub = 6, 44 << 20
    d_in = cp.generate(n, ub, seed=0xC0DE0909, zero_thresh=26, device=DEV)
    in_off, in_len = cp.uniform_layout(n, ub, device=DEV)
    slot = cp.encode_bound(ub)
    pk_off, pk_cap = cp.uniform_layout(n, slot, device=DEV)
    d_pk = torch.empty(n * slot, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
    d_out = torch.zeros(n * ub, dtype=torch.uint8, device=DEV)
    ulen = torch.zeros(n, dtype=torch.int64, device=DEV)
    ust = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
    torch.cuda.synchronize()
    assert (pst == 0).all().item() and int(plen.sum().item()) > 32768 * WIN
    assert (ust == 0).all().item() and torch.equal(ulen, in_len)
    assert torch.equal(d_out, d_in)


def test_failures_beyond_the_window_table_write_nothing():
    # as above (some units go to the serial decoder), with units cut one byte short
    # (UNEXPECTED_EOF) and slots 8 B short (OUT_OF_SPACE): their slots keep the sentinel
    n, ub = 6, 44 << 20
    d_in = cp.generate(n, ub, seed=0xC0DE090A, zero_thresh=26, device=DEV)
    in_off, in_len = cp.uniform_layout(n, ub, device=DEV)
    slot = cp.encode_bound(ub)
    pk_off, pk_cap = cp.uniform_layout(n, slot, device=DEV)
    d_pk = torch.empty(n * slot, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
    torch.cuda.synchronize()
    assert (pst == 0).all().item() and int(plen.sum().item()) > 32768 * WIN
    kind = [i % 3 for i in range(n)]  # 0 OK, 1 truncated, 2 slot too small
    cut = torch.tensor([1 if k == 1 else 0 for k in kind], dtype=torch.int64, device=DEV)
    short = torch.tensor([8 if k == 2 else 0 for k in kind], dtype=torch.int64, device=DEV)
    d_out = torch.full((n * ub,), 0xA5, dtype=torch.uint8, device=DEV)
    ulen = torch.zeros(n, dtype=torch.int64, device=DEV)
    ust = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_pk, pk_off, plen - cut, d_out, in_off, in_len - short, ulen, ust)
    torch.cuda.synchronize()
    for i, k in enumerate(kind):
        s = d_out[i * ub:(i + 1) * ub]
        if k == 0:
            assert ust[i].item() == cp.OK and ulen[i].item() == ub
            assert torch.equal(s, d_in[i * ub:(i + 1) * ub])
        else:
            assert ust[i].item() == (cp.UNEXPECTED_EOF if k == 1 else cp.OUT_OF_SPACE)
            assert ulen[i].item() == (0 if k == 1 else ub)
            assert (s == 0xA5).all().item(), (i, k, "failed unit wrote into its slot")
