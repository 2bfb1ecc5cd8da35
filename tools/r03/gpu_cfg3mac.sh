#!/bin/bash
# cfg3 many-chains MAC kernel with the 2-chunk whole-ring reload: LB 3 (148 VGPRs, m32) / LB 4 (128, spills, m42) vs base (1-chunk ring)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_cfg3mac
mkdir -p $O
TLSGPU_LIB=$R/tools/ab/m32/libtlsgpu.so timeout -k 10 300 python bench.py --config cfg3 --no-host-inclusive --no-open --no-derive --no-cpu > $O/check.json 2> $O/check.err || { tail -20 $O/check.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check.json'));print('check m32', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
bash tools/ab_bench.sh $O cfg3 3 base m32 m42 || exit 1
