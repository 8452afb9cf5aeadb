set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 120 python -u tools/eigh_probe.py > gpurun_out/r06c/eigh_probe.json 2>&1 &&
timeout -k 10 600 python -u tools/molecule_run.py --molecule porphyrin --kind xtda --nroots 20 --out gpurun_out/r06c/r06_porphyrin_xtda.json > gpurun_out/r06c/porph_xtda.log 2>&1 &&
timeout -k 10 600 python -u tools/molecule_run.py --molecule porphyrin --method 1 --out gpurun_out/r06c/r06_porphyrin_sfup_mc.json > gpurun_out/r06c/porph_mc.log 2>&1 &&
timeout -k 10 900 python -u tools/molecule_run.py --molecule c60- --tol 1e-8 --out gpurun_out/r06c/r06_c60_xsf_tol1e-8.json > gpurun_out/r06c/c60_tol8.log 2>&1
