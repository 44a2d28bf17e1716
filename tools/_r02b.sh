set -o pipefail
mkdir -p gpurun_out/r02k
bash tools/ab.sh nsref cur nsref cur
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "teacher or one_env or internals or variations" > gpurun_out/r02k/pytest.log 2>&1; echo pytest rc $?
tail -2 gpurun_out/r02k/pytest.log
timeout -k 10 300 python tools/stage_profile.py --steps 20 --out gpurun_out/r02k/stage_profile.json > gpurun_out/r02k/stage.log 2>&1
echo stage rc $?
