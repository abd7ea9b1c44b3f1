# r06q: the full GPU suite (with the slowest tests listed), the driver's bench under rocprofv3 and
# the PMC traffic passes at the round-6 head
set -o pipefail
NKV_PYTEST_ARGS="-x --durations=40" bash tools/gpu_round.sh r06q --pytest
