set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests > gpurun_out/g1_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/g1_tests.log; exit 1; }
tail -2 gpurun_out/g1_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-converge > gpurun_out/g1_b.json 2>gpurun_out/g1_b.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/g1_b.json'));print(d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['gemm_classes'].items()}, d['roofline'])"
