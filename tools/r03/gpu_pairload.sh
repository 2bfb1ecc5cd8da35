#!/bin/bash
# MAC (one-generation kernel, 2-chunk ring): both ring slots reloaded together (pairload) vs one per chunk
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_pairload
mkdir -p $O
TLSGPU_LIB=$R/tools/ab/pairload/libtlsgpu.so timeout -k 10 300 python bench.py --config cfg2 --no-host-inclusive --no-open --no-derive --no-cpu > $O/check.json 2> $O/check.err || { tail -20 $O/check.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check.json'));print('check pairload', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
bash tools/ab_bench.sh $O cfg2 3 base pairload || exit 1
