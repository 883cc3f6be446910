set -o pipefail
bash tools/gpu_final.sh r06d || exit 1
