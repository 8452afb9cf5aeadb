#!/bin/bash
# A/B with a FETCH_SIZE pass per variant (L2-miss bytes per kernel class)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
F=${FILE:-xt_gemm}
cp xtddft_amd/csrc/$F.hip /tmp/${F}_a.hip; cp xtddft_amd/_lib/libxtddft_amd.so /tmp/lib_a.so
for v in a ${VARIANTS:-b}; do
  if [ $v = a ]; then cp /tmp/${F}_a.hip xtddft_amd/csrc/$F.hip; cp /tmp/lib_a.so xtddft_amd/_lib/libxtddft_amd.so;
  else cp tools/ab/${F}_$v.hip xtddft_amd/csrc/$F.hip; cp tools/ab/lib_$v.so xtddft_amd/_lib/libxtddft_amd.so; fi
  timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-converge > gpurun_out/pab_$v.json 2>gpurun_out/pab.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/pab_$v.json'));print('$v', d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['gemm_classes'].items()})"
  mkdir -p gpurun_out/pab_$v
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pab_$v/FETCH_SIZE -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-converge > gpurun_out/pab_$v/FETCH_SIZE.log 2>&1 || exit 1
done
