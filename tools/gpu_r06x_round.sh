# r06x: the final round-6 pass: full GPU suite, the driver's bench under rocprofv3, PMC traffic
set -o pipefail
bash tools/gpu_round.sh r06x --pytest
