"""The kernel's fp64 sin / cos restatement (mj_envs_amd/csrc/aw_sincos64.h: Cody-Waite reduction
by pi/2 and fdlibm's published k_sin / k_cos kernels, used for the fp64 body frames) against libm,
compiled on the host from the same header: <= 1 ulp with fused multiply-adds (the kernel is built
with -ffp-contract=on on a target with FMA), <= 4 ulp without."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _fma_cpu():
    try:
        return " fma " in open("/proc/cpuinfo").read().replace("\n", " ")
    except OSError:
        return False


@pytest.mark.parametrize("fma", [False, True])
def test_sincos64_against_libm(tmp_path, fma):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    if fma and not _fma_cpu():
        pytest.skip("host CPU without FMA")
    exe = str(tmp_path / "sc")
    flags = ["-mfma", "-ffp-contract=fast"] if fma else ["-ffp-contract=off"]
    subprocess.run([cxx, "-O2", *flags, "-o", exe, os.path.join(HERE, "sincos64_check.cc")], check=True)
    ms, mc = map(float, subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split())
    bound = 1.0 if fma else 4.0
    assert ms <= bound and mc <= bound, (ms, mc)
