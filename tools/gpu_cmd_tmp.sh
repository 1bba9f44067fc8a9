set -e
export TMPDIR=/tmp
bash tools/round_end.sh r04_end
