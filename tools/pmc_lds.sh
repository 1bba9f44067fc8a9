#!/bin/bash
# LDS bank-conflict passes (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE per kernel) of a bench run.
# usage (GPU box): [PROG=tools/bench_full17.py] tools/pmc_lds.sh OUTDIR [bench args...]
set -e
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS \
  --output-format csv -d "$OUT" -o lds -- python3 ${PROG:-bench.py} "$@" > "$OUT/lds.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r['Kernel_Name'][:60]][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in tot.items():
    a = c.get('SQ_LDS_IDX_ACTIVE', 0)
    if a:
        print(f"{k:60s} conflict {c.get('SQ_LDS_BANK_CONFLICT',0):.3e} / active {a:.3e} = {c.get('SQ_LDS_BANK_CONFLICT',0)/a:.3f}  insts {c.get('SQ_INSTS_LDS',0):.3e}")
PY
