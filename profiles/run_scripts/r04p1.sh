set -o pipefail
export TMPDIR=/tmp
TAG=r04p tools/configs.sh c2 c4
