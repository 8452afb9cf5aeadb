#!/bin/bash
# SQ / GRBM counter passes over the bench's XC GEMM classes (one pass per counter
# group, each under its own limit; <= 8 SQ + 2 GRBM counters per pass).
#   BENCH_ARGS  bench.py arguments (default: headline, 1 step)
#   PASSES      space-separated pass names from the table below (default: all)
set -uo pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-sq}
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:-"--steps 1 --warmup 1 --no-cpu-baseline --no-converge"}
declare -A PMC
PMC[a]="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
PMC[b]="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT"
PMC[c]="SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES SQ_LEVEL_WAVES"
PMC[f]="FETCH_SIZE"
PMC[w]="WRITE_SIZE"
for p in ${PASSES:-a b c f w}; do
  timeout -k 10 240 rocprofv3 --pmc ${PMC[$p]} --kernel-trace --output-format csv -d "$OUT/$p" -o run -- python3 bench.py $ARGS > "$OUT/$p.log" 2>&1
  rc=$?
  echo "pass $p rc=$rc"
  [ $rc = 0 ] || exit $rc
done
