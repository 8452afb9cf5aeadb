# device Becke partition: device integral tests, then the porphyrin front end (kernel times)
set -o pipefail
mkdir -p gpurun_out/r06g19
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frontend.py > gpurun_out/r06g19/pytest.log 2>&1 || { tail -30 gpurun_out/r06g19/pytest.log; exit 1; }
tail -2 gpurun_out/r06g19/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06g19/prof -o run -- python3 -u $GRAFT_REPO_ROOT/tools/molecule_run.py --molecule porphyrin --scf-only > $GRAFT_REPO_ROOT/gpurun_out/r06g19/log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r06g19/log; exit 1; }
grep -E "^build|^scf" $GRAFT_REPO_ROOT/gpurun_out/r06g19/log | cut -c1-600
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r06g19/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:4]: print(round(float(r["TotalDurationNs"])/1e9,3), "s", r["Calls"], r["Name"][:90])
PY
