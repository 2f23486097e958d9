"""CPU: the C-ABI library builds, loads and exports every symbol declared in
include/pp2.h (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re

import pytest

from path_planning_2d_amd import _lib


def header_symbols():
    text = open(_lib.HEADER_PATH).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(pp2_\w+)\s*\(", text, re.M)))


def test_header_parsed():
    syms = header_symbols()
    assert "pp2_create" in syms and "pp2_loop_step" in syms
    assert len(syms) >= 30


def test_library_exports_header_symbols():
    lib = _lib.load()
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(_lib.SIGNATURES) == header_symbols()


def test_version_and_status_strings():
    lib = _lib.load()
    m = re.search(r"#define PP2_ABI_VERSION (\d+)", open(_lib.HEADER_PATH).read())
    assert m and int(m.group(1)) == _lib.PP2_ABI_VERSION
    assert lib.pp2_abi_version() == _lib.PP2_ABI_VERSION
    assert lib.pp2_status_string(0) == b"ok"
    assert lib.pp2_status_string(6) == b"RCCL error"


def test_errors_are_returned_not_fatal():
    """No device here: create must fail with a status, not exit()."""
    import numpy as np
    from path_planning_2d_amd import GridContext, Pp2Error
    g = np.zeros((4, 4), np.uint8)
    with pytest.raises(Pp2Error):
        GridContext(g, (1, 1), device=99)
    with pytest.raises(Pp2Error):
        _lib.call("pp2_create", ctypes.byref(ctypes.c_void_p()), 0, 0, 4,
                  g.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 0, 0,
                  ctypes.c_float(0.95))


def test_c_client_compiles_and_links(tmp_path):
    """examples/pp2_node_demo.c -- the POMDP node's sequence in plain C99 --
    compiles against include/pp2.h and links against the in-tree library."""
    import shutil
    import subprocess
    cc = shutil.which("cc") or shutil.which("gcc")
    if cc is None:
        pytest.skip("no C compiler")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib_dir = os.path.join(root, "path_planning_2d_amd")
    if not os.path.exists(os.path.join(lib_dir, "libpp2_hip.so")):
        pytest.skip("library not built")
    exe = tmp_path / "demo"
    subprocess.run([cc, "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(root, "include"),
                    "-o", str(exe), os.path.join(root, "examples", "pp2_node_demo.c"),
                    "-L", lib_dir, "-lpp2_hip"], check=True)
    assert exe.exists()
