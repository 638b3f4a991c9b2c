# Round-2 end: checkpoint (GPU suite, smoke, bench, rocprof passes) and the other BASELINE configs.
set -euo pipefail
bash tools/round_r02c.sh ${1:-r02s}
TAG=${1:-r02s}_configs bash tools/configs_r02.sh
