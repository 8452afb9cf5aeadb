set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06b/pytest.log 2>&1 &&
for c in C1 C5 C2; do timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 > gpurun_out/r06b/bench_$c.json 2> gpurun_out/r06b/bench_$c.err || exit 1; done &&
for c in C5 C2; do timeout -k 10 600 python -u bench.py --config $c --steps 5 --warmup 1 --cpu-converge on > gpurun_out/r06b/bench_${c}_cpuconv.json 2> gpurun_out/r06b/bench_${c}_cpuconv.err || exit 1; done
