"""The C-ABI library loads and exports every entry point include/adroit_wave.h declares
(no compute calls: this runs on the CPU-only build container)."""
import os
import re

from conftest import REPO


def declared_symbols():
    src = open(os.path.join(REPO, "include", "adroit_wave.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(aw_\w+)\s*\(", src, re.M)))


def test_header_declares_boundary():
    syms = declared_symbols()
    for s in ("aw_create", "aw_reset", "aw_step", "aw_get_state", "aw_set_state", "aw_status",
              "aw_destroy", "aw_last_error", "aw_task_eval", "aw_random_actions"):
        assert s in syms


def test_library_exports_all_symbols():
    import ctypes
    from mj_envs_amd import _native
    lib = _native.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
        assert isinstance(getattr(lib, s), ctypes._CFuncPtr)
    assert set(declared_symbols()) == set(_native.EXPORTS)


def test_no_cpu_fallback_in_product():
    """The product package must not import the oracle (test infrastructure)."""
    pkg = os.path.join(REPO, "mj_envs_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                txt = open(os.path.join(root, f)).read()
                assert "pyoracle" not in txt and "from oracle" not in txt, f
