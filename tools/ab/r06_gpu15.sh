# SQ counters of the integral kernel over the porphyrin front end
set -o pipefail
mkdir -p gpurun_out/r06g15
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06g15/pmc -o run -- python3 -u $GRAFT_REPO_ROOT/tools/molecule_run.py --molecule porphyrin --scf-only > $GRAFT_REPO_ROOT/gpurun_out/r06g15/log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r06g15/log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r06g15/pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys,collections
tot=collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_int_cart" in r["Kernel_Name"]:
        tot[r["Counter_Name"]]+=float(r["Counter_Value"])
for k,v in sorted(tot.items()): print(k, "%.4g" % v)
PY
