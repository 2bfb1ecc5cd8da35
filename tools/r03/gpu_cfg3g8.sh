#!/bin/bash
# cfg3: pair kernel with 8-block groups (whole-line loads and stores, 105 VGPRs) vs 4-block (base)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_cfg3g8
mkdir -p $O
TLSGPU_LIB=$R/tools/ab/gm8/libtlsgpu.so timeout -k 10 300 python bench.py --config cfg3 --no-host-inclusive --no-open --no-derive --no-cpu > $O/check.json 2> $O/check.err || { tail -20 $O/check.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check.json'));print('check gm8', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
bash tools/ab_bench.sh $O cfg3 3 base gm8 || exit 1
