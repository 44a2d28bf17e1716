set -e
timeout -k 10 120 python -u tools/rollout_dump.py /tmp/r06r_main.npz > gpurun_out/r06r_dump.log 2>&1
AW_LIB=mj_envs_amd/libadroit_hip_rsel0.so timeout -k 10 120 python -u tools/rollout_dump.py /tmp/r06r_rsel0.npz >> gpurun_out/r06r_dump.log 2>&1
AW_LIB=mj_envs_amd/libadroit_hip_kson.so timeout -k 10 120 python -u tools/rollout_dump.py /tmp/r06r_kson.npz >> gpurun_out/r06r_dump.log 2>&1
python - >> gpurun_out/r06r_dump.log <<'PY'
import numpy as np
a = np.load("/tmp/r06r_main.npz")
for other in ("rsel0", "kson"):
    b = np.load(f"/tmp/r06r_{other}.npz")
    for k in a.files:
        print("main vs", other, k, "bitwise equal" if np.array_equal(a[k], b[k]) else f"DIFFER max {np.abs(a[k]-b[k]).max():.3e}")
PY
bash tools/ab.sh rsel0 main kson > gpurun_out/r06r_ab_random.txt 2>&1
bash tools/ab.sh -p dapg rsel0 main kson > gpurun_out/r06r_ab_dapg.txt 2>&1
