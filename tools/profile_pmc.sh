#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass; gfx950 slot limits: SQ 8, TCC 4, GRBM 2) over a
# short bench run.  Usage (on the GPU box): [PROG=tools/bench_full17.py] tools/profile_pmc.sh OUTDIR [bench args...]
# Counters are collected in their own runs with --kernel-trace only (no sys/runtime trace).
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:---workload c3 --steps 2 --warmup 1 --no-cpu-baseline}
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
  "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_VALU_MFMA_COEXEC_CYCLES"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT" -o pass$i -- python3 ${PROG:-bench.py} $ARGS > "$OUT/pass$i.log" 2>&1
done
echo done
