#!/bin/bash
# Loop-body instruction mix of one kernel without the sin/cos large-argument fallback
# (MPCB_SC_FALLBACK=0, counting only).  usage: tools/isa_count.sh SOURCE.hip MANGLED_KERNEL [extra flags]
set -e
SRC=$(realpath $1); K=$2; shift 2
D=$(mktemp -d)
(cd $D && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -DMPCB_SC_FALLBACK=0 "$@" \
  -c $SRC -o x.o -save-temps 2>/dev/null)
python3 $(dirname $0)/isa_loop.py $D/*gfx950.s $K
grep -A12 "\.name:.*$K" $D/*gfx950.s | grep -E "vgpr_count|sgpr_spill|vgpr_spill" || true
rm -rf $D
