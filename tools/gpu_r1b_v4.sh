set -o pipefail
cd /root/repo
bash tools/gpu_r1b_v3.sh && bash tools/gpu_r1b.sh
