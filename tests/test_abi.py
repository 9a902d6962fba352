"""The C ABI boundary (CPU only, no compute): libcordagpu.so loads, exports every entry
point include/cordagpu.h declares, struct layouts match, and without a GPU it fails loudly
(no CPU fallback)."""
import ctypes
import os

import numpy as np
import pytest

from corda_amd import _lib
from corda_amd import batch as B


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    syms = _lib.declared_symbols()
    assert len(syms) >= 17
    assert [s for s in syms if not hasattr(L, s)] == []
    assert L.cg_abi_version() == 2
    assert b"gfx950" in L.cg_build_info()


def test_struct_layouts_match_header():
    src = open(_lib.HEADER_PATH).read()
    assert "} cg_key;            /* 16 bytes */" in src
    assert "} cg_item;           /* 32 bytes */" in src
    assert B.KEY_DTYPE.itemsize == 16 and B.ITEM_DTYPE.itemsize == 32
    assert B.TX_DTYPE.itemsize == 24 and B.COMPONENT_DTYPE.itemsize == 16
    assert [B.KEY_DTYPE.fields[f][1] for f in ("off", "len", "scheme", "fmt")] == [0, 8, 10, 11]
    assert [B.ITEM_DTYPE.fields[f][1] for f in ("sig_off", "msg_off", "msg_len", "key_idx", "sig_len")] == \
        [0, 8, 16, 20, 24]


def test_status_codes_match_header():
    src = open(_lib.HEADER_PATH).read()
    for name, code in (("CG_VALID", 0), ("CG_INVALID", 1), ("CG_SIG_MALFORMED", 2), ("CG_KEY_INVALID", 3),
                       ("CG_UNSUPPORTED", 4), ("CG_EMPTY", 5), ("CG_NOT_RUN", 255)):
        assert f"{name} = {code}" in src
    from oracle import corda
    assert (corda.VALID, corda.INVALID, corda.SIG_MALFORMED, corda.KEY_INVALID, corda.UNSUPPORTED, corda.EMPTY) == \
        (B.VALID, B.INVALID, B.SIG_MALFORMED, B.KEY_INVALID, B.UNSUPPORTED, B.EMPTY)


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="CPU-only behaviour")
def test_no_gpu_fails_loudly():
    L = _lib.lib()
    assert L.cg_device_count() == 0
    h = ctypes.c_void_p()
    cfg = _lib.cg_config(0, 0, 0, 0)
    rc = L.cg_open(ctypes.byref(h), ctypes.byref(cfg))
    assert rc != 0 and not h.value
    assert len(_lib.last_error()) > 0
    from corda_amd.engine import Engine
    with pytest.raises(_lib.EngineUnavailable):
        Engine(0)


def test_null_ctx_is_an_argument_error():
    L = _lib.lib()
    st = np.zeros(4, dtype=np.uint8)
    assert L.cg_verify_batch(None, None, 0, None, 0, None, 0, 0, None, None) == -1
    assert L.cg_verify_items_device(None, None, 0, None, 1, None, 0, 0, st.ctypes.data_as(ctypes.c_void_p),
                                    None) == -1
