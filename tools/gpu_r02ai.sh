#!/bin/bash
# r02ai: 3DES split-address round (dessplit) vs base on cfg5, with one oracle-checked run; DES microbench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02ai
mkdir -p $O
cd $R
TLSGPU_LIB=$R/tools/ab/dessplit/libtlsgpu.so timeout -k 10 300 python bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu --no-host-inclusive --no-open --no-derive > $O/check.json 2> $O/check.err || { tail -5 $O/check.err; exit 1; }
python -c "import json;d=json.load(open('$O/check.json'));print('dessplit checked', d['value'], d['bit_exact'])"
bash tools/ab_bench.sh gpurun_out/r02ai cfg5 3 base dessplit || exit 1
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/des_layout_microbench.hip -o $O/dmb.bin 2>/dev/null && timeout -k 10 120 $O/dmb.bin 256
echo done
