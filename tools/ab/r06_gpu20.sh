# where the porphyrin SCF spends its wall time (cProfile, top cumulative entries)
set -o pipefail
mkdir -p gpurun_out/r06g20
timeout -k 10 600 python -u -m cProfile -o gpurun_out/r06g20/scf.prof tools/molecule_run.py --molecule porphyrin --scf-only > gpurun_out/r06g20/log 2>&1 || { tail -20 gpurun_out/r06g20/log; exit 1; }
python - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/r06g20/scf.prof")
p.sort_stats("cumulative").print_stats(35)
PY
