# round-6 GPU step: fp16x3 entry traces; layer4-entry PMC traffic, shipped vs the 2 x 4 XCD split (6:48)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 6 --variant 58 --launch 5 9 --precision fp16x3 > $O/trace_x3entries.log 2>&1 || exit 1
TAG=r06g tools/gpu_check.sh fetch:base || exit 1
TAG=r06g FWD_ARGS="--variant 6:48" tools/gpu_check.sh fetch:split48
