#!/bin/bash
# small-batch XC shapes: tests, nvec sweep, headline bench + converge
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_parity.py > gpurun_out/sm_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sm_tests.log; exit 1; }
tail -2 gpurun_out/sm_tests.log
timeout -k 10 200 python -u tools/nvec_sweep.py --out gpurun_out/sm_nv.json > gpurun_out/sm_nv.log 2>&1 || exit 1
grep nvec gpurun_out/sm_nv.log
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline > gpurun_out/sm_b.json 2>gpurun_out/sm_b.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/sm_b.json'));print(d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['gemm_classes'].items()}, d['converge'])"
