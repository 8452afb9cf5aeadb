#!/bin/bash
# same-box A/B/... of source files: the tree as uploaded (a) against variants v, whose
# versions of FILE (a .hip under csrc) and of the EXTRA csrc files (e.g. xt_internal.h) are
# tools/ab/<stem>_<v>.<ext>, with the prebuilt library tools/ab/lib_<v>.so
# (VARIANTS="b c ..."); bench lines alternate a b c ... over ROUNDS rounds
set -o pipefail
mkdir -p gpurun_out /tmp/ab_a
F=${FILE:-xt_xcm}
FILES="$F.hip ${EXTRA:-}"
for f in $FILES; do cp xtddft_amd/csrc/$f /tmp/ab_a/$f; done
cp xtddft_amd/_lib/libxtddft_amd.so /tmp/ab_a/lib.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in a ${VARIANTS:-b}; do
    for f in $FILES; do
      if [ $v = a ]; then cp /tmp/ab_a/$f xtddft_amd/csrc/$f; else cp tools/ab/${f%.*}_$v.${f##*.} xtddft_amd/csrc/$f; fi
    done
    if [ $v = a ]; then cp /tmp/ab_a/lib.so xtddft_amd/_lib/libxtddft_amd.so; else cp tools/ab/lib_$v.so xtddft_amd/_lib/libxtddft_amd.so; fi
    timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-converge ${BENCH_ARGS:-} > gpurun_out/ab_$v$r.json 2>gpurun_out/ab.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_$v$r.json'));print('$v', d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['gemm_classes'].items()})"
  done
done
for f in $FILES; do cp /tmp/ab_a/$f xtddft_amd/csrc/$f; done
cp /tmp/ab_a/lib.so xtddft_amd/_lib/libxtddft_amd.so
