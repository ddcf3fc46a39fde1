"""Generate tests/golden/zig_vectors.json — Zig-rule golden vectors.

Nothing in the reference pins the encoder's bytes, so these
vectors are produced by the C oracle (oracle/packed_oracle.c, a restatement of
message.zig:200-271) and accepted only where the independent Python
restatement (tests/pyref.py) produces identical bytes. Decoder outcomes are
additionally pinned by the reference's own fixture pairs (tests/golden/fixtures).

Run:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle  # noqa: E402
import pyref  # noqa: E402

FIX = os.path.join(HERE, "fixtures")


def w(*bs):
    assert len(bs) == 8
    return bytes(bs)


FULL = w(1, 2, 3, 4, 5, 6, 7, 8)
ONEZ = w(1, 2, 0, 4, 5, 6, 7, 8)  # exactly one zero byte (C++ would extend a literal run with it)
MIX = w(0, 9, 0, 0, 7, 0, 0, 1)
ZERO = bytes(8)


def synthetic_cases():
    cases = {
        "empty": b"",
        "one_zero_word": ZERO,
        "one_full_word": FULL,
        "one_mixed_word": MIX,
        "full_then_onezero": FULL + ONEZ,        # Zig ends the literal run; C++ would not
        "full_onezero_full": FULL + ONEZ + FULL,
        "zero_run_255": ZERO * 255,
        "zero_run_256": ZERO * 256,
        "zero_run_257": ZERO * 257,
        "zero_run_512": ZERO * 512,
        "zero_run_513": ZERO * 513,
        "literal_run_255": FULL * 255,
        "literal_run_256": FULL * 256,
        "literal_run_257": FULL * 257,
        "literal_run_600": FULL * 600,
        "zero_full_alternating": (ZERO + FULL) * 64,
        "full_mixed_alternating": (FULL + ONEZ) * 64,  # worst case 9 B/word
        "walking_ones": b"".join(struct.pack("<Q", 1 << k) for k in range(64)),
        "tag_sweep": b"".join(bytes((0xA5 if (t >> k) & 1 else 0) for k in range(8)) for t in range(256)),
        "zero_literal_zero": ZERO * 3 + FULL * 5 + ZERO * 300 + FULL * 2,
    }
    rng = random.Random(0x5EED)
    for p in (0.1, 0.5, 0.9):
        data = bytes(0 if rng.random() < p else rng.randrange(1, 256) for _ in range(1024))
        cases[f"random_1KiB_p{p}"] = data
    # a framed 64-segment message of 1 KiB i.i.d. p=0.5 segments (config C1)
    segs = [bytes(0 if rng.random() < 0.5 else rng.randrange(1, 256) for _ in range(1024)) for _ in range(64)]
    cases["framed_64x1KiB_p0.5"] = pyref.frame(segs)
    return cases


def main():
    vectors = []
    for name in ("binary", "segmented", "fixture_single.bin", "fixture_far.bin"):
        data = open(os.path.join(FIX, name), "rb").read()
        vectors.append(("fixture:" + name, data))
    for name, data in synthetic_cases().items():
        vectors.append((name, data))

    out = {"generator": "tests/golden/make_golden.py",
           "rules": "Zig packPacked, message.zig:200-271 (NOT canonical C++ capnp)",
           "vectors": []}
    for name, data in vectors:
        st, packed = oracle.pack(data)
        assert st == 0, name
        assert packed == pyref.pack(data), f"oracle and pyref disagree on {name}"
        st, back = oracle.unpack(packed)
        assert st == 0 and back == data, name
        rec = {"name": name, "unpacked_len": len(data), "packed_len": len(packed),
               "unpacked_sha256": hashlib.sha256(data).hexdigest(),
               "packed_sha256": hashlib.sha256(packed).hexdigest()}
        if not name.startswith("fixture:"):
            rec["unpacked_hex"] = data.hex()
        rec["packed_hex"] = packed.hex()
        out["vectors"].append(rec)
    path = os.path.join(HERE, "zig_vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {path}: {len(out['vectors'])} vectors")


if __name__ == "__main__":
    main()
