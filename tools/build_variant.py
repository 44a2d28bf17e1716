"""Build an experimental variant of the HIP library (hammer NV=33 only) for A/B timing.

    python tools/build_variant.py NAME [-DFLAG ...]   -> mj_envs_amd/libadroit_hip_NAME.so
    AW_LIB=mj_envs_amd/libadroit_hip_NAME.so python bench.py ...   (on the GPU box)
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from __graft_entry__ import HIPCC_FLAGS, HIP_SRC  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(REPO, "mj_envs_amd", f"libadroit_hip_{name}.so")
subprocess.run(["/opt/rocm/bin/hipcc", *HIPCC_FLAGS, "-DAW_ONLY_TASK=0", *flags, "-o", out, HIP_SRC], check=True)
print(out)
