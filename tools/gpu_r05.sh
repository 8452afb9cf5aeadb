#!/bin/bash
# round 5: the GPU suite (TESTS / K select a subset), then optional bench lines (BENCH="C2 H ...")
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05}
timeout -k 10 ${LIMIT:-900} python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread ${TESTS:-tests} ${K:+-k "$K"} > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${T}_tests.log; [ $rc = 0 ] || exit $rc
for c in ${BENCH:-}; do
  timeout -k 10 ${BLIMIT:-400} python -u bench.py --config $c ${BARGS:-} > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/${T}_bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/${T}_bench_$c.json')); print('$c', d['value'], d.get('verify',{}).get('rel_err'), d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
done
for m in ${MOLS:-}; do
  timeout -k 10 ${MLIMIT:-600} python -u tools/molecule_run.py --molecule $m > gpurun_out/${T}_mol_$m.log 2>&1 || { echo "molecule $m failed"; tail -5 gpurun_out/${T}_mol_$m.log; exit 1; }
  tail -1 gpurun_out/${T}_mol_$m.log | cut -c1-400
done
