"""CPU checks of the C-ABI boundary: librx.so builds for gfx950, loads, and exports every entry
point declared in include/rx.h. No compute call (no GPU here)."""
import ctypes
import os

from tests.rxpkg import rx


def test_library_exports_every_header_symbol():
    if not os.path.exists(rx.LIB_PATH):
        rx.build()
    lib = ctypes.CDLL(rx.LIB_PATH)
    syms = rx.header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, f"missing exports: {missing}"


def test_status_strings():
    if not os.path.exists(rx.LIB_PATH):
        rx.build()
    assert rx.lib().rx_status_string(rx.RX_ERR_NAN).decode().startswith("NaN")


def test_gfx950_code_object_present():
    if not os.path.exists(rx.LIB_PATH):
        rx.build()
    data = open(rx.LIB_PATH, "rb").read()
    assert b"gfx950" in data
