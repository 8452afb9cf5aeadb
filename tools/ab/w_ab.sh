# same-box A/B of small-O XC kernel choices on C5 / C2 (environment variants); parity first
set -o pipefail
mkdir -p gpurun_out/w
XT_W_KERNEL=1 XT_W_PERS=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "not reference" > gpurun_out/w/tests.log 2>&1 || { tail -30 gpurun_out/w/tests.log; exit 1; }
echo "parity pers: $(tail -1 gpurun_out/w/tests.log)"
XT_M_RV0=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "not reference" > gpurun_out/w/tests2.log 2>&1 || { tail -30 gpurun_out/w/tests2.log; exit 1; }
echo "parity rv0: $(tail -1 gpurun_out/w/tests2.log)"
for r in 1 2; do
for cfg in C5 C2; do
  for v in "base" "XT_W_KERNEL=1" "XT_W_KERNEL=1 XT_W_PERS=4" "XT_W_KERNEL=1 XT_W_PERS=8" "XT_M_RV0=1"; do
    env $([ "$v" = base ] || echo $v) timeout -k 10 200 python -u bench.py --config $cfg --steps 30 --no-converge --no-cpu-baseline > gpurun_out/w/b.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/w/b.json'));print('$cfg', '$v', d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['gemm_classes'].items()})"
  done
done
done
