# same-box A/B of environment variants: VARS="base|A=1|A=2 B=3" (| separated), NVECS, CFG
set -o pipefail
mkdir -p gpurun_out/env
IFS='|' read -ra VV <<< "${VARS:-base}"
for r in 1 2; do
for nv in ${NVECS:-1 3 20}; do
  st=5; [ $nv -lt 10 ] && st=15
  for v in "${VV[@]}"; do
    env $([ "$v" = base ] || echo $v) timeout -k 10 200 python -u bench.py --config ${CFG:-H} --nvec $nv --steps $st --no-converge --no-cpu-baseline > gpurun_out/env/b.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/env/b.json'));print('nvec $nv', '$v', d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['gemm_classes'].items()})"
  done
done
done
