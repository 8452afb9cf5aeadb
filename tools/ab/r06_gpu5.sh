set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_qc.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06d/pytest.log 2>&1 &&
for c in C2 C5 H; do timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r06d/bench_$c.json 2> gpurun_out/r06d/bench_$c.err || exit 1; done &&
TAG=r06d/sqC2 PASSES=b BENCH_ARGS="--config C2 --steps 2 --warmup 1 --no-cpu-baseline --no-converge" bash tools/profile_sq.sh &&
timeout -k 10 900 python -u tools/molecule_run.py --molecule c60- --tol 1e-8 --out gpurun_out/r06d/r06_c60_xsf_tol1e-8.json > gpurun_out/r06d/c60_tol8.log 2>&1
