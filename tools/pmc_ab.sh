#!/bin/bash
# PMC passes (tools/pmc_kernels.sh) of one config for several library builds: "base" = the
# product library, any other name = tools/ab/<name>/libtlsgpu.so (tools/build_ab.sh).
#   bash tools/pmc_ab.sh <outdir> <config> <variant>...      -> <outdir>/pmc_<variant>.json
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; CFG=$2
shift 2
mkdir -p $O
cd $R
for v in "$@"; do
  if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so; fi
  timeout -k 10 600 bash tools/pmc_kernels.sh $CFG $O/pmc_$v > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -20 $O/pmc_$v.log; exit 1; }
  cp $R/profiles/pmc_$CFG.json $O/pmc_$v.json
  python3 -c "
import json;d=json.load(open('$O/pmc_$v.json'))
for k,v in sorted(d['kernels'].items(), key=lambda kv: -kv[1].get('duration_ms',0))[:4]:
    print('$v', k[:40], 'ms', round(v.get('duration_ms',0),3), 'valu', v.get('SQ_INSTS_VALU'), 'lds', v.get('SQ_INSTS_LDS'), 'hbm', v.get('hbm_bytes'), 'clk', v.get('clock_ghz'), 'ldsbusy', v.get('lds_busy'), 'valu/simd/cyc', v.get('valu_inst_per_simd_cycle'))
print('$v', 'seal call hbm', d['seal_call_hbm_bytes'])"
done
unset TLSGPU_LIB
git -C $R checkout -q -- profiles/pmc_$CFG.json 2>/dev/null || true
