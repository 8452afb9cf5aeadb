set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 1500 python -u -m pytest tests/test_gpu_molecule.py tests/test_gpu_solver.py tests/test_gpu_drivers.py tests/test_gpu_fullsize.py -x -v --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/r06a/pytest.log 2>&1 &&
for c in C1 C5 C2; do timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 > gpurun_out/r06a/bench_$c.json 2> gpurun_out/r06a/bench_$c.err || exit 1; done
