export CFGS="32 16 32 1 8"
bash tools/experiments/gpu_r03_seamtune.sh
