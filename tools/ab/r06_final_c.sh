# round-6 final (c): the BASELINE-scale molecules end to end with the late front end
set -o pipefail
mkdir -p gpurun_out/r06fc
timeout -k 10 400 python -u tools/molecule_run.py --molecule porphyrin --out gpurun_out/r06fc/r06_porphyrin_sfup.json > gpurun_out/r06fc/porph.log 2>&1 || { tail -20 gpurun_out/r06fc/porph.log; exit 1; }
grep -E "^build|^scf|^solve|verify" gpurun_out/r06fc/porph.log | cut -c1-400
timeout -k 10 700 python -u tools/molecule_run.py --molecule c60- --kind xtda --nroots 20 --no-oracle --out gpurun_out/r06fc/r06_c60_xtda.json > gpurun_out/r06fc/c60.log 2>&1 || { tail -20 gpurun_out/r06fc/c60.log; exit 1; }
grep -E "^build|^scf|^solve|verify" gpurun_out/r06fc/c60.log | cut -c1-400
