#!/bin/bash
# same-box A/B/... of one source file: the tree as uploaded (a) against variants
# tools/ab/<file>_<v>.hip with prebuilt libraries tools/ab/lib_<v>.so (VARIANTS="b c ...");
# bench lines alternate a b c ... over ROUNDS rounds
set -o pipefail
mkdir -p gpurun_out
F=${FILE:-xt_xcm}
cp xtddft_amd/csrc/$F.hip /tmp/${F}_a.hip; cp xtddft_amd/_lib/libxtddft_amd.so /tmp/lib_a.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in a ${VARIANTS:-b}; do
    if [ $v = a ]; then cp /tmp/${F}_a.hip xtddft_amd/csrc/$F.hip; cp /tmp/lib_a.so xtddft_amd/_lib/libxtddft_amd.so;
    else cp tools/ab/${F}_$v.hip xtddft_amd/csrc/$F.hip; cp tools/ab/lib_$v.so xtddft_amd/_lib/libxtddft_amd.so; fi
    timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-converge ${BENCH_ARGS:-} > gpurun_out/ab_$v$r.json 2>gpurun_out/ab.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_$v$r.json'));print('$v', d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['gemm_classes'].items()})"
  done
done
