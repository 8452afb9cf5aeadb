#!/bin/bash
# A/B of the rho-forward variants on one box: tests, headline bench, nvec sweep per variant.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_variants.py -k "barrier_free or xc_kernel" > gpurun_out/w2_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/w2_tests.log; exit 1; }
tail -2 gpurun_out/w2_tests.log
for v in 1 2 1 2; do
  XT_W_VARIANT=$v timeout -k 10 200 python -u bench.py --steps 5 --no-cpu-baseline --no-converge > gpurun_out/w2_b$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/w2_b$v.json'));print('variant $v', d['value'], d['ms_per_step'], d['gemm_classes']['xc_forward_w']['ms_per_step'])"
done
for v in 1 2; do
  XT_W_VARIANT=$v timeout -k 10 200 python -u tools/nvec_sweep.py --out gpurun_out/w2_nv$v.json > gpurun_out/w2_nv$v.log 2>&1 || exit 1
  echo "variant $v"; cat gpurun_out/w2_nv$v.log | grep nvec
done
