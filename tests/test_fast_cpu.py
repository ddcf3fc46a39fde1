"""oracle/packed_fast.c (bench.py's CPU baseline, a word-at-a-time port of message.zig:88-271)
against the checker (oracle/packed_oracle.c): same statuses, lengths and bytes for every
density, ragged unit sizes, units that fill a literal or zero run past 256 words, truncated and
corrupted packed streams, and slots too small (where the port hands the unit to the checker)."""
import numpy as np
import pytest

import oracle


def _layout(sizes):
    off = np.zeros(len(sizes) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(np.asarray(sizes, dtype=np.uint64))
    return off


def _units(rng, n, p_zero):
    sizes = rng.integers(0, 700, n) * 8
    sizes[:4] = [0, 8, 4096, 8 * 600]
    data = rng.integers(1, 256, int(sizes.sum()), dtype=np.uint8)
    data[rng.random(len(data)) < p_zero] = 0
    # long zero runs and long literal runs (> 256 words) in a few units
    off = _layout(sizes)
    if sizes[3]:
        b = int(off[3])
        data[b:b + 8 * 300] = 0
    if sizes[2]:
        b = int(off[2])
        data[b:b + 8 * 280] = rng.integers(1, 256, 8 * 280, dtype=np.uint8)
    return data, sizes


def _same(a, b, lens_a, lens_b, off):
    assert np.array_equal(lens_a, lens_b)
    for i in range(len(lens_a)):
        s = int(off[i])
        assert np.array_equal(a[s:s + int(lens_a[i])], b[s:s + int(lens_b[i])]), f"unit {i}"


@pytest.mark.parametrize("p_zero", [0.0, 0.1, 0.5, 0.9, 1.0])
def test_fast_pack_unpack_match_checker(p_zero):
    rng = np.random.default_rng(int(p_zero * 100) + 7)
    data, sizes = _units(rng, 400, p_zero)
    in_off = _layout(sizes)
    slots = (sizes // 8) * 10 + 16
    pk_off = _layout(slots)
    ref, ref_len, ref_st = oracle.pack_batch(data, in_off, pk_off)
    got, got_len, got_st = oracle.fast_pack_batch(data, in_off, pk_off)
    assert np.array_equal(ref_st, got_st) and (ref_st == 0).all()
    _same(ref, got, ref_len, got_len, pk_off)
    dense = np.concatenate([ref[int(pk_off[i]):int(pk_off[i]) + int(ref_len[i])] for i in range(len(sizes))])
    d_off = _layout(ref_len)
    r2, r2_len, r2_st = oracle.unpack_batch(dense, d_off, in_off)
    g2, g2_len, g2_st = oracle.fast_unpack_batch(dense, d_off, in_off)
    assert np.array_equal(r2_st, g2_st) and (r2_st == 0).all()
    _same(r2, g2, r2_len, g2_len, in_off)
    assert np.array_equal(g2[:len(data)], data)


def test_fast_tight_slots_and_bad_streams_match_checker():
    rng = np.random.default_rng(11)
    data, sizes = _units(rng, 300, 0.5)
    in_off = _layout(sizes)
    # pack slots from 0 to the exact size: the port hands these units to the checker
    ref_full, ref_len, _ = oracle.pack_batch(data, in_off, _layout((sizes // 8) * 10 + 16))
    tight = np.maximum(ref_len.astype(np.int64) - rng.integers(-2, 3, len(sizes)), 0).astype(np.uint64)
    t_off = _layout(tight)
    a, a_len, a_st = oracle.pack_batch(data, in_off, t_off)
    b, b_len, b_st = oracle.fast_pack_batch(data, in_off, t_off)
    assert np.array_equal(a_st, b_st) and np.array_equal(a_len, b_len)
    ok = a_st == 0
    _same(a, b, np.where(ok, a_len, 0), np.where(ok, b_len, 0), t_off)
    # truncated and corrupted packed units, and output slots a word short
    units = []
    for i in range(len(sizes)):
        pk = ref_full[int(_layout((sizes // 8) * 10 + 16)[i]):][:int(ref_len[i])].copy()
        k = i % 4
        if k == 1 and len(pk):
            pk = pk[:rng.integers(0, len(pk))]
        elif k == 2 and len(pk):
            pk[rng.integers(0, len(pk))] = rng.integers(0, 256)
        units.append(pk)
    p_off = _layout([len(u) for u in units])
    packed = np.concatenate(units) if units else np.zeros(0, np.uint8)
    caps = sizes.copy()
    caps[3::4] = np.maximum(caps[3::4].astype(np.int64) - 8, 0).astype(caps.dtype)
    c_off = _layout(caps)
    r, r_len, r_st = oracle.unpack_batch(packed, p_off, c_off)
    g, g_len, g_st = oracle.fast_unpack_batch(packed, p_off, c_off)
    assert np.array_equal(r_st, g_st) and np.array_equal(r_len, g_len)
    assert (r_st != 0).any() and (r_st == 0).any()
    ok = r_st == 0
    _same(r, g, np.where(ok, r_len, 0), np.where(ok, g_len, 0), c_off)
