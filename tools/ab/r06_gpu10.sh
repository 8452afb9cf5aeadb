# small-O rho-forward tail split: parity (variants + tail-split test), then C2 / C5 bench lines
set -o pipefail
mkdir -p gpurun_out/r06g10
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_variants.py -k "tail_split or variants" > gpurun_out/r06g10/pytest.log 2>&1 || { tail -30 gpurun_out/r06g10/pytest.log; exit 1; }
tail -3 gpurun_out/r06g10/pytest.log
for c in C2 C5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --no-cpu-baseline --no-converge > gpurun_out/r06g10/bench_$c.json 2> gpurun_out/r06g10/bench_$c.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r06g10/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['gemm_classes'].items()})"
done
