# same-box A/B of the stored-exchange stream shapes, run with a temporary XT_SK_MID knob in
# sk_shape (xt_exch.hip; 0: the 160-row image for every M > 48, the old rule) -- the knob
# is not in the committed kernel
set -o pipefail
mkdir -p gpurun_out/sk
for v in 0 1 0 1; do
  XT_SK_MID=$v timeout -k 10 300 python -u tools/nvec_sweep.py --nvecs 20,30,40,80 --out gpurun_out/sk/H_$v.json > gpurun_out/sk/H_$v.log 2>&1 || exit 1
  python -c "
import json
for r in json.load(open('gpurun_out/sk/H_$v.json')): print('H mid=$v', r['nvec'], r['ms'], r['classes'].get('mo_exchange_stored'))"
  XT_SK_MID=$v timeout -k 10 300 python -u bench.py --config C4 --steps 3 --no-cpu-baseline > gpurun_out/sk/C4_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sk/C4_$v.json').read().strip().splitlines()[-1]);print('C4 mid=$v', d['value'], d['ms_per_step'], d['gemm_classes']['mo_exchange_stored']['ms_per_step'], d['converge']['wall_s'], d['converge']['iterations'])"
done
