set -o pipefail
export TMPDIR=/tmp
TAG=r04p tools/configs.sh c1 c3
