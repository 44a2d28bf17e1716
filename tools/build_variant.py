"""Build an experimental variant of the HIP library (all four tasks, the split build) for A/B timing.

    python tools/build_variant.py NAME [-DFLAG ...]   -> mj_envs_amd/libadroit_hip_NAME.so
    AW_LIB=mj_envs_amd/libadroit_hip_NAME.so python bench.py ...   (on the GPU box)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from __graft_entry__ import build_hip  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(REPO, "mj_envs_amd", f"libadroit_hip_{name}.so")
build_hip(out, tuple(flags))
print(out)
