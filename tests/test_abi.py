"""C-ABI checks that need no GPU: the library loads, exports every symbol that
include/capnp_packed.h declares, and refuses to compute without a device
(there is no CPU fallback in the product path)."""
import ctypes
import os
import re
import subprocess

import pytest

import capnp_packed as cp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "capnp_packed.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(capnp_packed_\w+)\s*\(", text)))


def test_header_declares_expected_surface():
    names = declared_functions()
    for must in ("capnp_packed_encode", "capnp_packed_decode", "capnp_packed_decoded_size",
                 "capnp_packed_encode_batch", "capnp_packed_decode_batch", "capnp_packed_encode_bound"):
        assert must in names


def test_library_exports_every_declared_symbol():
    L = cp.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert set(declared_functions()) == set(cp.SIGNATURES), "ctypes signature table out of sync with header"


def test_exports_are_c_symbols():
    out = subprocess.check_output(["nm", "-D", "--defined-only", cp.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for name in declared_functions():
        assert name in exported, f"{name} not exported unmangled"


def test_version_and_status_names():
    assert cp.lib().capnp_packed_abi_version() == 2
    names = [cp.lib().capnp_packed_status_name(i).decode() for i in range(8)]
    assert names == ["Ok", "InvalidMessageSize", "UnexpectedEof", "Overflow", "OutOfSpace",
                     "InvalidArgument", "DeviceError", "NoDevice"]
    assert cp.encode_bound(4096) == 5120 and cp.encode_bound(0) == 0
    # Reader.readPackedMessage errors (reader.zig:84-156)
    names = [cp.lib().capnp_packed_status_name(i).decode() for i in range(8, 14)]
    assert names == ["EndOfStream", "InvalidSegmentCount", "SegmentCountLimitExceeded", "MessageTooLarge",
                     "InvalidPackedMessage", "TruncatedMessage"]
    for st in range(14):
        if st:
            assert cp._ERRORS[st].status == st


def test_read_message_argument_validation_without_device():
    n, used = ctypes.c_size_t(5), ctypes.c_size_t(5)
    assert cp.lib().capnp_packed_read_message(None, 8, None, 0, ctypes.byref(n), ctypes.byref(used)) == \
        cp.INVALID_ARGUMENT
    assert n.value == 0 and used.value == 0
    assert cp.lib().capnp_packed_read_message(b"\x00\x00", 2, None, 0, None, ctypes.byref(used)) == \
        cp.INVALID_ARGUMENT


def test_gfx950_code_object_present():
    blob = open(cp.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob  # the offload bundle carries a gfx950 code object


def test_argument_validation_without_device():
    n = ctypes.c_size_t(123)
    assert cp.lib().capnp_packed_encode(None, 8, None, 0, ctypes.byref(n)) == cp.INVALID_ARGUMENT
    assert n.value == 0
    assert cp.lib().capnp_packed_encode(b"1234567", 7, None, 0, ctypes.byref(n)) == cp.INVALID_MESSAGE_SIZE


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="checks the no-device behaviour")
def test_no_cpu_fallback_without_device():
    with pytest.raises(cp.NoDevice):
        cp.pack_packed(bytes(16))
    with pytest.raises(cp.NoDevice):
        cp.unpack_packed(b"\x00\x00")


def header_statuses():
    text = open(HEADER).read()
    return {name: int(v) for name, v in re.findall(r"CAPNP_PACKED_(\w+)\s*=\s*(\d+)", text)
            if name != "ABI_VERSION" and not name.startswith("DECODER_")}


def test_status_tables_agree():
    # header enum == Python constants / error classes == library names == Zig binding enum
    st = header_statuses()
    assert len(st) == 23 and sorted(st.values()) == list(range(23))
    for name, v in st.items():
        assert getattr(cp, name) == v, name
        if v:
            assert cp._ERRORS[v].status == v
        assert cp.lib().capnp_packed_status_name(v).decode() != "Unknown"
    zig = open(os.path.join(REPO, "zig", "packed_ffi.zig")).read()
    zig_enum = dict((n, int(v)) for n, v in re.findall(r"^\s+(\w+) = (\d+),$", zig, flags=re.M))
    assert {k.lower(): v for k, v in st.items()} == zig_enum


def test_decoder_selection_round_trips():
    # capnp_packed_set_decoder is a process-wide knob (no device needed to set it)
    prev = cp.set_decoder("words")
    assert cp.set_decoder("twopass") == "words"
    with cp.decoder("words"):
        assert cp.set_decoder("words") == "words"
    assert cp.set_decoder(prev) == "twopass"
    assert cp.decoder_available("auto") and cp.decoder_available("words")
    # the fused / streaming decoders were removed in round 5
    for gone in ("fused", "stream"):
        assert not cp.decoder_available(gone)
        assert cp.lib().capnp_packed_set_decoder(cp.DECODERS[gone]) == cp.INVALID_ARGUMENT
    assert cp.lib().capnp_packed_set_decoder(7) == cp.INVALID_ARGUMENT
    assert cp.set_all_or_nothing(True) is False
    assert cp.set_all_or_nothing(False) is True


def test_zig_binding_declares_only_header_symbols():
    zig = open(os.path.join(REPO, "zig", "packed_ffi.zig")).read()
    externs = set(re.findall(r'extern "capnp_packed" fn (capnp_packed_\w+)', zig))
    assert externs <= set(declared_functions()), externs - set(declared_functions())
    assert "capnp_packed_validate_batch" in externs


def test_validate_argument_errors_without_device():
    L = cp.lib()
    st = L.capnp_packed_validate_batch(None, None, None, 0, 512, 1 << 23, 64, None, None, None)
    assert st == cp.OK  # n = 0: nothing to do
    st = L.capnp_packed_validate_batch(None, None, None, 4, 512, 1 << 23, 64, None, None, None)
    assert st == cp.INVALID_ARGUMENT


def test_frame_connections_argument_errors_without_device():
    L = cp.lib()
    nf = ctypes.c_uint32(7)
    args = [None, 0, None, None, 0, None, None, 0, None, None, None, 0, None, None]
    assert L.capnp_packed_frame_connections(*args, ctypes.byref(nf)) == cp.OK and nf.value == 0  # no connections
    assert L.capnp_packed_frame_connections(*args, None) == cp.INVALID_ARGUMENT
    import numpy as np
    off = np.array([0, 6], dtype=np.uint64)
    ln = np.array([4, 4], dtype=np.uint64)  # connection 1's bytes run past in_bytes = 8
    guess = np.full(2, 8192, dtype=np.uint64)
    buf = np.zeros(8, dtype=np.uint8)
    fr = np.zeros(64, dtype=np.uint8)
    t64 = np.zeros(4, dtype=np.uint64)
    t32 = np.zeros(4, dtype=np.uint32)
    st32 = np.zeros(2, dtype=np.int32)
    st = L.capnp_packed_frame_connections(buf.ctypes.data, 8, off.ctypes.data, ln.ctypes.data, 2, guess.ctypes.data,
                                          fr.ctypes.data, 64, t64.ctypes.data, t64.ctypes.data, t32.ctypes.data, 4,
                                          t64.ctypes.data, st32.ctypes.data, ctypes.byref(nf))
    assert st == cp.INVALID_ARGUMENT
