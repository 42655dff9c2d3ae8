"""librbhip.so loads and exports every entry point include/rbhip.h declares;
argument validation works without a GPU (no compute calls here)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "rbhip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rb_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    path = os.path.join(PKG, "rbhip", "librbhip.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)
    from rbhip import _lib
    return _lib.load(path)


def test_header_declares_the_boundary():
    fns = header_functions()
    for f in ("rb_world_create", "rb_step", "rb_set_state", "rb_get_state", "rb_get_contacts",
              "rb_kat_impulse", "rb_shard_step", "rb_last_error"):
        assert f in fns


def test_library_exports_every_header_symbol(lib):
    path = os.path.join(PKG, "rbhip", "librbhip.so")
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, f"declared in include/rbhip.h but not exported: {missing}"


def test_python_binding_covers_header(lib):
    from rbhip import _lib
    assert sorted(_lib.SIGNATURES) == header_functions()


def test_scene_desc_layout_matches_header():
    """ctypes mirror of rb_scene_desc: field offsets as a C compiler lays it out."""
    from rbhip import _lib
    d = _lib.SceneDesc
    assert d.kind.offset == 40 and d.gravity.offset == 80 and C.sizeof(d) == 104


def test_version_and_errors_without_device(lib):
    from rbhip import _lib
    assert b"gfx950" in lib.rb_version()
    # argument validation happens before any device call
    h = C.c_void_p()
    rc = lib.rb_world_create(C.byref(h), None)
    assert rc == -22 and b"null" in lib.rb_last_error()
    d = _lib.SceneDesc()
    d.n_bodies = 0
    assert lib.rb_world_create(C.byref(h), C.byref(d)) == -22
    assert lib.rb_step(None, 1, 0.01, 0.5, 0.5, 0.0) == -22
    assert lib.rb_kat_impulse(0, 7, 1, None, None) == -22


def test_product_path_has_no_oracle_dependency():
    """The shipped package must never import or link the oracle."""
    for dirpath, _, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".h", ".cpp")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "liboracle" not in txt and "from oracle" not in txt and "import oracle" not in txt, f
    path = os.path.join(PKG, "rbhip", "librbhip.so")
    if os.path.exists(path):
        out = subprocess.run(["ldd", path], capture_output=True, text=True).stdout
        assert "oracle" not in out


def test_world_requires_library_loudly(tmp_path):
    from rbhip import _lib
    with pytest.raises(RuntimeError, match="not built"):
        _lib._lib, saved = None, _lib._lib
        try:
            _lib.load(str(tmp_path / "missing.so"))
        finally:
            _lib._lib = saved
    assert np is not None


def test_kernels_do_not_spill():
    """Every kernel of librbhip.so compiles for gfx950 with no scratch (a
    spill or an address-taken local in the step kernels costs latency on
    every step)."""
    out = subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc"), "resource-usage"],
                         capture_output=True, text=True, check=True).stdout
    names = re.findall(r"Function Name: (\S+)", out)
    scratch = [int(v) for v in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", out)]
    assert names and len(names) == len(scratch)
    spilled = [n for n, s in zip(names, scratch) if s]
    assert not spilled, f"kernels with scratch: {spilled}"
