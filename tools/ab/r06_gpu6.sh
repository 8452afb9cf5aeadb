set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_variants.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06e/pytest.log 2>&1 &&
for c in C2 C5 H C3; do timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-converge > gpurun_out/r06e/bench_$c.json 2> gpurun_out/r06e/bench_$c.err || exit 1; done &&
TAG=r06e/sqC2 PASSES=b BENCH_ARGS="--config C2 --steps 2 --warmup 1 --no-cpu-baseline --no-converge" bash tools/profile_sq.sh &&
TAG=r06e/sqC5 PASSES=b BENCH_ARGS="--config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-converge" bash tools/profile_sq.sh
