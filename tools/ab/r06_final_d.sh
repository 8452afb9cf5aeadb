# round-6 final (d): bench lines of the large configs again, now that this round's PMC summary holds
# them (roofline.traffic); CONFIGS picks the set
set -o pipefail
mkdir -p gpurun_out/r06fd
for c in ${CONFIGS:-H C3 C3mc}; do
  mkdir -p gpurun_out/r06fd/$c
  timeout -k 10 500 python3 -u bench.py --config $c > gpurun_out/r06fd/$c/bench.log 2>&1 || { tail -5 gpurun_out/r06fd/$c/bench.log; exit 1; }
  tail -c 300 gpurun_out/r06fd/$c/bench.log; echo
done
