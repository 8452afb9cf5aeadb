# forward U tile A/B at the small configurations: default (cfg 8: 128 x 128 BK 16, rows on the
# SIMDs, two blocks per CU) vs cfg 9 (BK 32, one block per CU) vs cfg 5
set -o pipefail
mkdir -p gpurun_out/ucfg
for c in C2 C5; do
  for r in 1 2; do
    for f in 0 9 5; do
      if [ $f = 0 ]; then unset XT_GEMM_U_CFG; else export XT_GEMM_U_CFG=$f; fi
      timeout -k 10 300 python -u bench.py --config $c --steps 5 --no-cpu-baseline --no-converge > gpurun_out/ucfg/b.json 2> gpurun_out/ucfg/b.err || exit 1
      python -c "import json;d=json.load(open('gpurun_out/ucfg/b.json'));print('$c cfg $f', d['value'], d['ms_per_step'], d['gemm_classes']['xc_forward_u']['ms_per_step'])"
    done
  done
done
unset XT_GEMM_U_CFG
