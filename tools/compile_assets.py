"""Compile the reference's Adroit MJCF into the committed model tables (models/*.npz).

Run in the build container (where /root/reference exists):
    python tools/compile_assets.py [--assets DIR]
The GPU box has no /root/reference; it loads the committed .npz tables.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mj_envs_amd.mjcf import compile_mjcf  # noqa: E402
from mj_envs_amd.tasks import MODEL_DIR, TASKS  # noqa: E402

DEFAULT_ASSETS = "/root/reference/mj_envs_vision/hand_manipulation_suite/assets"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--assets", default=os.environ.get("ADROIT_ASSETS", DEFAULT_ASSETS))
    args = ap.parse_args()
    os.makedirs(MODEL_DIR, exist_ok=True)
    for spec in TASKS.values():
        m = compile_mjcf(os.path.join(args.assets, spec.xml))
        out = os.path.join(MODEL_DIR, spec.xml.replace(".xml", ".npz"))
        m.save_npz(out)
        print(spec.env_id, m.dims, "->", out)


if __name__ == "__main__":
    main()
