#!/bin/bash
# same-box A/B of one source file: the tree as uploaded (A) against tools/ab/<file>_b.hip with
# its prebuilt library tools/ab/lib_b.so (B); bench lines alternate A B A B
set -o pipefail
mkdir -p gpurun_out
F=${FILE:-xt_xcm}
cp xtddft_amd/csrc/$F.hip /tmp/${F}_a.hip; cp xtddft_amd/_lib/libxtddft_amd.so /tmp/lib_a.so
for r in 1 2; do
  for v in a b; do
    if [ $v = a ]; then cp /tmp/${F}_a.hip xtddft_amd/csrc/$F.hip; cp /tmp/lib_a.so xtddft_amd/_lib/libxtddft_amd.so;
    else cp tools/ab/${F}_b.hip xtddft_amd/csrc/$F.hip; cp tools/ab/lib_b.so xtddft_amd/_lib/libxtddft_amd.so; fi
    timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-converge ${BENCH_ARGS:-} > gpurun_out/ab_$v$r.json 2>gpurun_out/ab.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_$v$r.json'));print('$v', d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['gemm_classes'].items()})"
  done
done
