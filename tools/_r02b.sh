set -o pipefail
mkdir -p gpurun_out/r02l
bash tools/ab.sh regoffd cur regoffd cur
timeout -k 10 300 python tools/stage_profile.py --steps 20 --out gpurun_out/r02l/stage_profile.json > gpurun_out/r02l/stage.log 2>&1
echo stage rc $?
