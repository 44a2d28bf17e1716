#!/bin/bash
# Bitwise A/B of library variants (run through gpurun): bash tools/ab_bitwise.sh TAG variant...
# Deterministic rollouts (tools/rollout_dump.py) of main and of each mj_envs_amd/libadroit_hip_<variant>.so
# compared array for array, then tools/ab.sh under the random and DAPG policies.  Dumps stay in /tmp
# on the box (they exceed gpurun_out's size cap); logs go to gpurun_out/TAG_*.
set -e
TAG=$1; shift
timeout -k 10 120 python -u tools/rollout_dump.py /tmp/${TAG}_main.npz > gpurun_out/${TAG}_dump.log 2>&1
for v in "$@"; do
  AW_LIB=mj_envs_amd/libadroit_hip_$v.so timeout -k 10 120 python -u tools/rollout_dump.py /tmp/${TAG}_$v.npz >> gpurun_out/${TAG}_dump.log 2>&1
done
python - "$TAG" "$@" >> gpurun_out/${TAG}_dump.log <<'PY'
import sys
import numpy as np
tag = sys.argv[1]
a = np.load(f"/tmp/{tag}_main.npz")
for other in sys.argv[2:]:
    b = np.load(f"/tmp/{tag}_{other}.npz")
    for k in a.files:
        print("main vs", other, k, "bitwise equal" if np.array_equal(a[k], b[k]) else f"DIFFER max {np.abs(a[k]-b[k]).max():.3e}")
PY
bash tools/ab.sh main "$@" > gpurun_out/${TAG}_ab_random.txt 2>&1
bash tools/ab.sh -p dapg main "$@" > gpurun_out/${TAG}_ab_dapg.txt 2>&1
