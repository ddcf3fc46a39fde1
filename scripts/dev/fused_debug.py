"""Decode a few batches through decode_batch and report per-unit mismatches vs the oracle."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "capnp-zig_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np, torch
import capnp_packed as cp, oracle

def run(units, tag):
    n = len(units)
    dev = torch.device("cuda", 0)
    lens = [len(u) for u in units]
    off = np.zeros(n, dtype=np.int64); off[1:] = np.cumsum(lens)[:-1]
    buf = np.frombuffer(b"".join(units) + bytes(64), dtype=np.uint8)
    d_in = torch.from_numpy(buf.copy()).to(dev)
    in_off = torch.from_numpy(off).to(dev); in_len = torch.tensor(lens, dtype=torch.int64, device=dev)
    exp = [oracle.unpack(u) for u in units]
    caps = [max(8, len(e[1])) for e in exp]
    ooff = np.zeros(n, dtype=np.int64); ooff[1:] = np.cumsum(caps)[:-1]
    d_out = torch.zeros(int(sum(caps)) + 64, dtype=torch.uint8, device=dev)
    o_off = torch.from_numpy(ooff).to(dev); o_cap = torch.tensor(caps, dtype=torch.int64, device=dev)
    olen = torch.zeros(n, dtype=torch.int64, device=dev); st = torch.full((n,), -7, dtype=torch.int32, device=dev)
    cp.decode_batch(d_in, in_off, in_len, d_out, o_off, o_cap, olen, st)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy(); olen = olen.cpu().numpy(); st = st.cpu().numpy()
    bad = 0
    for i in range(n):
        es, eb = exp[i]
        got = out[ooff[i]:ooff[i] + olen[i]].tobytes() if st[i] == 0 else b""
        if st[i] != es or (es == 0 and got != eb):
            if bad < 8:
                print(f"{tag} unit {i}: P={lens[i]} exp st={es} len={len(eb)} | got st={st[i]} len={olen[i]}"
                      + (f" firstdiff={next((k for k in range(min(len(got),len(eb))) if got[k]!=eb[k]), None)}" if es == 0 and st[i] == 0 else ""))
            bad += 1
    print(f"{tag}: {n} units, {bad} bad")

fx = os.path.join(HERE, "..", "..", "tests", "golden", "fixtures")
run([open(os.path.join(fx, "packed"), "rb").read()] * 4, "fixture")
for thr in (128, 26, 230):
    h = oracle.generate(256, 4096, seed=0xC0DE0003, zero_thresh=thr)
    units = [oracle.pack(h[i * 4096:(i + 1) * 4096].tobytes())[1] for i in range(256)]
    run(units, f"thr{thr}")
