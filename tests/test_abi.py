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


def test_ctypes_structs_match_header_layout(tmp_path):
    """The Python mirror's structs have the C header's field offsets (gcc on include/rx.h)."""
    import subprocess
    structs = {"rx_mesh_desc": rx.MeshDesc, "rx_host_comm": rx.HostComm, "rx_cfg": rx.Cfg}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rx.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    inc = os.path.dirname(rx.HEADER)
    subprocess.run(["gcc", "-I", inc, str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l.strip()}
    for cname, py in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_python_enums_match_header():
    """rx_field / rx_kernel order in the Python mirror is the header's."""
    import re
    txt = open(rx.HEADER).read()

    def names(enum, prefix):
        body = re.search(r"typedef enum \{([^{}]*)\}\s*%s;" % enum, txt).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        out = []
        for tok in body.split(","):
            tok = tok.strip().split("=")[0].strip()
            if tok:
                out.append(tok[len(prefix):])
        return [n for n in out if n != "COUNT"]

    assert names("rx_field", "RX_F_") == rx.FIELDS
    assert names("rx_kernel", "RX_K_") == rx.KERNELS
