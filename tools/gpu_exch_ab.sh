#!/bin/bash
# Stored-exchange row shapes: the variant tests, then headline benches at nvec 1/4/8/16 and
# C3 with the 16/32-row A images (XT_SKINNY_SMALL=1, default) and without (=0).
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread > gpurun_out/var.log 2>&1; rc=$?; tail -2 gpurun_out/var.log; [ $rc = 0 ] || exit $rc
for n in 1 4 8 16; do for sm in 0 1; do
  XT_SKINNY_SMALL=$sm timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-converge --nvec $n > gpurun_out/ex_${n}_$sm.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['gemm_classes']['mo_exchange_stored']['ms_per_step'])" gpurun_out/ex_${n}_$sm.log "nvec=$n small=$sm"
done; done
for sm in 0 1; do
  XT_SKINNY_SMALL=$sm timeout -k 10 200 python -u bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-converge > gpurun_out/ex_C3_$sm.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['gemm_classes']['mo_exchange_stored']['ms_per_step'])" gpurun_out/ex_C3_$sm.log "C3 small=$sm"
done
