# same-box A/B of the point-kernel variants (XT_POINT_B=0: k_xc_point; 1..4: k_xc_point_b
# with ds_bpermute / DPP exchanges and one / two batches in flight); parity first
set -o pipefail
mkdir -p gpurun_out/pt
for b in ${PARITY:-2 4}; do
  XT_POINT_B=$b timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_molecule.py -k "not reference" > gpurun_out/pt/tests$b.log 2>&1 || { tail -30 gpurun_out/pt/tests$b.log; exit 1; }
  echo "parity XT_POINT_B=$b: $(tail -1 gpurun_out/pt/tests$b.log)"
done
for r in 1 2; do
for cfg in ${CFGS:-C5 C2 H}; do
  st=5; [ $cfg != H ] && st=30
  for b in ${VARS:-0 1 2 3 4}; do
    XT_POINT_B=$b timeout -k 10 200 python -u bench.py --config $cfg --steps $st --no-converge --no-cpu-baseline > gpurun_out/pt/$cfg.$b.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/pt/$cfg.$b.json'));print('$cfg', $b, d['value'], d['ms_per_step'])"
  done
done
done
