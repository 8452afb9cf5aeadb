# round-6 final (b): bench lines, kernel stats and FETCH / WRITE passes for the configs the
# late small-O change touches (C1, C2, C5)
set -o pipefail
TAG=r06fb CONFIGS="C1 C2 C5" bash tools/evidence.sh
