#!/bin/bash
# Round evidence in one GPU call: the default bench line (N = 1, CPU baseline and
# Davidson included), then tools/profile_r01.sh's rocprofv3 passes (trace + stats,
# FETCH_SIZE, WRITE_SIZE).  Summarise afterwards with tools/parse_prof.py.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-round}
mkdir -p "$OUT"
timeout -k 10 500 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; tail -1 "$OUT/bench.log"; [ $rc = 0 ] || exit $rc
PROF_TAG=${TAG:-round}/prof tools/profile_r01.sh
