#!/bin/bash
# quick check after a kernel change: XC variant tests + parity + headline bench + nvec sweep
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-q}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_parity.py > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-converge > gpurun_out/${T}_b$r.json 2>gpurun_out/${T}_b.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/${T}_b$r.json'));print(d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['gemm_classes'].items()}, d['roofline']['frac'])"
done
if [ -n "$SWEEP" ]; then timeout -k 10 200 python -u tools/nvec_sweep.py --nvecs 1,2,3,4,5,6,8,10,12 --out gpurun_out/${T}_nv.json > gpurun_out/${T}_nv.log 2>&1 && grep nvec gpurun_out/${T}_nv.log; fi
