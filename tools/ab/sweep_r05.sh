set -o pipefail
mkdir -p gpurun_out/sw
timeout -k 10 200 python -u tools/nvec_sweep.py --nao 128 --nclosed 11 --nvecs 1,8,20,40,80 --out gpurun_out/sw/n128.json > gpurun_out/sw/n128.log 2>&1 &&
timeout -k 10 200 python -u tools/nvec_sweep.py --nao 256 --nclosed 24 --nvecs 1,8,20,40,80 --out gpurun_out/sw/n256.json > gpurun_out/sw/n256.log 2>&1 &&
timeout -k 10 250 python -u tools/nvec_sweep.py --nao 512 --nclosed 49 --nvecs 1,8,20,40,80 --out gpurun_out/sw/n512.json > gpurun_out/sw/n512.log 2>&1 &&
timeout -k 10 400 python -u tools/nvec_sweep.py --nvecs 1,8,20,40,80 --out gpurun_out/sw/n1000.json > gpurun_out/sw/n1000.log 2>&1
