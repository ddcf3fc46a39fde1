"""The small-unit kernels (encode_small_kernel / decode_small_kernel):
units of at most 64 words (encode) or 512 packed bytes into a slot of at most 8 KiB
(decode) are coded one per lane. These tests hit their state machines directly:
- every output alignment (dense, odd offsets) with canary bytes around each slot: the
  packed bytes equal the oracle's (message.zig:200-271) and nothing outside a slot changes;
- literal runs whose count byte lands in an earlier, already written 16-B chunk (the
  patch path), zero runs of every length up to 64 words, runs at unit ends;
- OUT_OF_SPACE with slots one byte short (required length reported, nothing past the slot
  written), InvalidMessageSize and misaligned units mixed into the same batch;
- decode of the same units from dense unaligned packed bytes, truncated units
  (UnexpectedEof), short output slots (OUT_OF_SPACE), misaligned output slots;
- a batch mixing small, mid and long units, so the three classes run together.
"""
import numpy as np
import pytest

import capnp_packed as cp
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"
CANARY = 0xA5


def make_units(rng, n, max_words=64):
    units = []
    for i in range(n):
        w = int(rng.integers(0, max_words + 1))
        kind = i % 6
        words = []
        for j in range(w):
            r = rng.random()
            if kind == 0:  # long literal runs (count byte patched after its chunk is written)
                v = int(rng.integers(1, 256, 8, dtype=np.uint8).view(np.uint64)[0]) if r < 0.9 else 0
            elif kind == 1:  # zero runs
                v = 0 if r < 0.85 else int(rng.integers(1, 1 << 63))
            elif kind == 2:  # alternating runs
                v = 0 if (j // 3) % 2 else int(rng.integers(1, 256, 8, dtype=np.uint8).view(np.uint64)[0])
            else:  # mixed bytes
                b = rng.integers(0, 256, 8, dtype=np.uint8)
                b[rng.random(8) < 0.5] = 0
                v = int(b.view(np.uint64)[0])
            words.append(v)
        units.append(np.array(words, dtype=np.uint64).tobytes())
    return units


def pack_layout(units, rng, slack=16):
    """Inputs 8-aligned back to back; output slots at odd offsets with canary gaps."""
    in_off, pos = [], 0
    for u in units:
        in_off.append(pos)
        pos += len(u)
    blob = b"".join(units)
    exp = [oracle.pack(u)[1] for u in units]
    out_off, caps, p = [], [], 0
    for e in exp:
        p += int(rng.integers(1, slack))  # gap of canaries, any alignment
        out_off.append(p)
        caps.append(len(e))
        p += len(e)
    return blob, in_off, exp, out_off, caps, p + slack


def t64(x):
    return torch.tensor(x, dtype=torch.int64, device=DEV)


def test_encode_small_alignment_and_canaries():
    rng = np.random.default_rng(0x5A11)
    units = make_units(rng, 4000)
    blob, in_off, exp, out_off, caps, total = pack_layout(units, rng)
    d_in = torch.from_numpy(np.frombuffer(blob or b"\0", dtype=np.uint8).copy()).to(DEV)
    d_out = torch.full((total,), CANARY, dtype=torch.uint8, device=DEV)
    n = len(units)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    st = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, t64(in_off), t64([len(u) for u in units]), d_out, t64(out_off), t64(caps), plen, st)
    torch.cuda.synchronize()
    assert (st == 0).all().item()
    assert plen.cpu().tolist() == [len(e) for e in exp]
    h = d_out.cpu().numpy()
    mask = np.zeros(total, dtype=bool)
    for i, e in enumerate(exp):
        assert h[out_off[i]:out_off[i] + len(e)].tobytes() == e, f"unit {i}"
        mask[out_off[i]:out_off[i] + len(e)] = True
    assert (h[~mask] == CANARY).all(), "bytes outside the slots changed"


def test_encode_small_out_of_space_and_errors():
    rng = np.random.default_rng(0x5A12)
    units = [u for u in make_units(rng, 600) if u]
    blob, in_off, exp, out_off, caps, total = pack_layout(units, rng)
    caps = [c - 1 if i % 3 == 0 else c for i, c in enumerate(caps)]  # one byte short
    lens = [len(u) for u in units]
    for i in range(1, len(units), 7):
        lens[i] -= 3  # InvalidMessageSize
    d_in = torch.from_numpy(np.frombuffer(blob + b"\0" * 16, dtype=np.uint8).copy()).to(DEV)
    offs = list(in_off)
    for i in range(2, len(units), 11):
        offs[i] += 4  # misaligned word side: InvalidArgument
    d_out = torch.full((total,), CANARY, dtype=torch.uint8, device=DEV)
    n = len(units)
    plen = torch.full((n,), -1, dtype=torch.int64, device=DEV)
    st = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, t64(offs), t64(lens), d_out, t64(out_off), t64(caps), plen, st)
    torch.cuda.synchronize()
    st_h, pl_h, h = st.cpu().numpy(), plen.cpu().numpy(), d_out.cpu().numpy()
    for i in range(n):
        if offs[i] != in_off[i]:
            assert st_h[i] == cp.INVALID_ARGUMENT and pl_h[i] == 0
        elif lens[i] % 8:
            assert st_h[i] == cp.INVALID_MESSAGE_SIZE and pl_h[i] == 0
        elif caps[i] < len(exp[i]):
            assert st_h[i] == cp.OUT_OF_SPACE and pl_h[i] == len(exp[i])
        else:
            assert st_h[i] == cp.OK and h[out_off[i]:out_off[i] + caps[i]].tobytes() == exp[i]
    mask = np.zeros(total, dtype=bool)
    for i in range(n):
        mask[out_off[i]:out_off[i] + caps[i]] = True
    assert (h[~mask] == CANARY).all(), "bytes past a slot changed"


def test_decode_small_dense_truncated_and_short():
    rng = np.random.default_rng(0x5A13)
    units = make_units(rng, 3000)
    packed = [oracle.pack(u)[1] for u in units]
    # dense packed stream, then damage: truncate some units by one byte
    P = [len(p) for p in packed]
    cut = [i for i in range(len(units)) if i % 9 == 4 and P[i] > 0]
    for i in cut:
        P[i] -= 1
    off, pos = [], 0
    for p in packed:
        off.append(pos)
        pos += len(p)
    d_pk = torch.from_numpy(np.frombuffer(b"".join(packed) + b"\0" * 16, dtype=np.uint8).copy()).to(DEV)
    n = len(units)
    caps = [len(u) for u in units]
    short = [i for i in range(n) if i % 13 == 6 and caps[i] >= 8]
    for i in short:
        caps[i] -= 8
    o_off, q = [], 0
    for c in caps:
        q += 8 * int(rng.integers(1, 3))
        o_off.append(q)
        q += c
    d_out = torch.full((q + 16,), CANARY, dtype=torch.uint8, device=DEV)
    ulen = torch.full((n,), -1, dtype=torch.int64, device=DEV)
    st = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_pk, t64(off), t64(P), d_out, t64(o_off), t64(caps), ulen, st)
    torch.cuda.synchronize()
    st_h, ul_h, h = st.cpu().numpy(), ulen.cpu().numpy(), d_out.cpu().numpy()
    for i in range(n):
        est, ref = oracle.unpack(packed[i][:P[i]])
        if est != oracle.OK:
            assert st_h[i] == cp.UNEXPECTED_EOF and ul_h[i] == 0, i
        elif len(ref) > caps[i]:
            assert st_h[i] == cp.OUT_OF_SPACE and ul_h[i] == len(ref), i
        else:
            assert st_h[i] == cp.OK and ul_h[i] == len(ref), i
            assert h[o_off[i]:o_off[i] + len(ref)].tobytes() == ref, i
    mask = np.zeros(len(h), dtype=bool)
    for i in range(n):
        mask[o_off[i]:o_off[i] + caps[i]] = True
    assert (h[~mask] == CANARY).all(), "bytes past an output slot changed"


def test_decode_small_misaligned_slot():
    u = np.arange(1, 9, dtype=np.uint64).tobytes()
    p = oracle.pack(u)[1]
    d_pk = torch.from_numpy(np.frombuffer(p, dtype=np.uint8).copy()).to(DEV)
    d_out = torch.zeros(128, dtype=torch.uint8, device=DEV)
    ulen = torch.full((2,), -1, dtype=torch.int64, device=DEV)
    st = torch.full((2,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_pk, t64([0, 0]), t64([len(p), len(p)]), d_out, t64([0, 68]), t64([64, 64]), ulen, st)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [cp.OK, cp.INVALID_ARGUMENT]
    assert d_out[:64].cpu().numpy().tobytes() == u


def test_mixed_classes_roundtrip():
    rng = np.random.default_rng(0x5A14)
    sizes = rng.choice([8, 64, 512, 520, 2048, 4096, 4104, 40960, 200000], size=3000,
                       p=[.3, .2, .1, .05, .1, .1, .05, .07, .03]).astype(np.int64)
    sizes = sizes // 8 * 8
    U = int(sizes.sum())
    d_in = cp.generate(1, U, seed=0x5A15, zero_thresh=128, device=DEV)
    ln = torch.from_numpy(sizes).to(DEV)
    in_off = torch.zeros_like(ln)
    in_off[1:] = torch.cumsum(ln, 0)[:-1]
    cap = (ln // 8) * 10
    pk_off = torch.zeros_like(ln)
    pk_off[1:] = torch.cumsum(cap, 0)[:-1]
    d_pk = torch.empty(int(cap.sum().item()), dtype=torch.uint8, device=DEV)
    n = len(sizes)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, in_off, ln, d_pk, pk_off, cap, plen, pst)
    d_out = torch.empty(U, dtype=torch.uint8, device=DEV)
    ulen = torch.zeros(n, dtype=torch.int64, device=DEV)
    ust = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, ln, ulen, ust)
    torch.cuda.synchronize()
    assert (pst == 0).all().item() and (ust == 0).all().item()
    assert torch.equal(ulen, ln) and torch.equal(d_out, d_in)
    h_in, h_pk = d_in.cpu().numpy(), d_pk.cpu().numpy()
    io, po, pl = in_off.cpu().numpy(), pk_off.cpu().numpy(), plen.cpu().numpy()
    for i in range(0, n, 17):
        e = oracle.pack(h_in[io[i]:io[i] + sizes[i]].tobytes())[1]
        assert h_pk[po[i]:po[i] + pl[i]].tobytes() == e, i
