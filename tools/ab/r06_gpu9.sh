set -o pipefail
mkdir -p gpurun_out/r06_final_ev/C1 gpurun_out/r06_final_ev/C2 gpurun_out/r06_final_ev/C5
for c in C1 C2 C5; do timeout -k 10 400 python -u bench.py --config $c > gpurun_out/r06_final_ev/$c/bench.log 2>&1 || exit 1; done &&
for c in C2 C5; do timeout -k 10 600 python -u bench.py --config $c --steps 5 --warmup 1 --cpu-converge on > gpurun_out/r06_final_ev/$c/bench_cpuconv.log 2>&1 || exit 1; done &&
TAG=r06_final_sq/C2 PASSES="a b c" BENCH_ARGS="--config C2 --steps 2 --warmup 1 --no-cpu-baseline --no-converge" bash tools/profile_sq.sh &&
TAG=r06_final_sq/C5 PASSES="a b c" BENCH_ARGS="--config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-converge" bash tools/profile_sq.sh
