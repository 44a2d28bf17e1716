set -o pipefail
bash tools/ab.sh base nochg c0 c2 cur base nochg c0
