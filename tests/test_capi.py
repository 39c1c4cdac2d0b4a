"""The C-ABI library builds, loads without a GPU and exports every symbol the public
header declares (no compute calls here)."""
import ctypes
import glob
import os
import re

import pytest

from perseus_amd import _lib, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        syms |= set(re.findall(r"\b(pa_[a-z0-9_]+)\s*\(", txt))
    return syms


def test_header_declares_entry_points():
    s = declared_symbols()
    for need in ("pa_detector_create", "pa_detector_forward", "pa_detector_destroy", "pa_proj_linearize",
                 "pa_dyn_linearize", "pa_cv_linearize", "pa_last_error"):
        assert need in s


def test_library_exports_every_declared_symbol():
    path = build.build(verbose=False)
    L = ctypes.CDLL(path)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert set(_lib._SIGS) >= declared_symbols(), declared_symbols() - set(_lib._SIGS)


def test_version_and_error_string_without_gpu():
    L = _lib.lib()
    assert b"gfx950" in L.pa_version()
    assert isinstance(L.pa_last_error(), bytes)


def test_bad_arguments_fail_loudly_without_touching_the_gpu():
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.pa_detector_create(None, 0, 4, 8, 256, 256, ctypes.byref(h))
    assert rc == -1 and b"null weights" in L.pa_last_error()
    rc = L.pa_detector_create(ctypes.c_void_p(8), 16, 4, 8, 128, 128, ctypes.byref(h))
    assert rc == -1 and b"256x256" in L.pa_last_error()
    with pytest.raises(_lib.PerseusError):
        _lib.check(L.pa_dyn_linearize(1, None, None, None, None, 0.1, 7, None, None, None, None, None, None, None,
                                      None), "dyn")


def test_gfx950_code_object_present():
    data = open(build.LIB, "rb").read()
    assert b"gfx950" in data


def test_traj_args_struct_layout_matches_header(tmp_path):
    """The ctypes mirror of pa_traj_args has the C compiler's field offsets."""
    names = [f[0] for f in _lib.TrajArgs._fields_]
    src = tmp_path / "off.c"
    body = "".join(f'  printf("%zu\\n", offsetof(pa_traj_args, {n}));\n' for n in names)
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "perseus_amd.h"\nint main(void){\n'
                   + body + '  printf("%zu\\n", sizeof(pa_traj_args));\n  return 0;\n}\n')
    exe = tmp_path / "off"
    import subprocess
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    want = [getattr(_lib.TrajArgs, n).offset for n in names] + [ctypes.sizeof(_lib.TrajArgs)]
    assert got == want


def test_trajectory_rejects_bad_shapes_without_gpu():
    L = _lib.lib()
    a = _lib.TrajArgs()
    a.T, a.L, a.n_kp = 1, 0, 8
    assert L.pa_trajectory_linearize(ctypes.byref(a), None) == -1
    assert b"L=0" in L.pa_last_error()
    assert L.pa_trajectory_linearize(None, None) == -1
