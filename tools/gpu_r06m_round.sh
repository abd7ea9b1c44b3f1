# r06m: product rotation bit-identical to the pre-round-6 one, then the full GPU suite, the driver's
# bench under rocprofv3 and the PMC traffic passes
set -o pipefail
mkdir -p gpurun_out/r06m
timeout -k 10 200 python3 tools/check_variant_rotate.py rot_old base > gpurun_out/r06m/check_rot.log 2>&1 && \
bash tools/gpu_round.sh r06m --pytest
