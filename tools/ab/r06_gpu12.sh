# kernel-time breakdown of the porphyrin front end (integrals, Cholesky, SCF)
set -o pipefail
mkdir -p gpurun_out/r06g12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06g12/prof -o run -- python3 -u $GRAFT_REPO_ROOT/tools/molecule_run.py --molecule porphyrin --scf-only > $GRAFT_REPO_ROOT/gpurun_out/r06g12/log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r06g12/log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r06g12/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:15]: print(round(float(r["TotalDurationNs"])/1e9,3), "s", r["Calls"], r["Name"][:90])
PY
