export CFGS="32 16 32 1 8"
bash tools/gpu_r03_seamtune.sh
