#!/bin/bash
# One gpurun call = a list of steps on one MI355X, each under its own time limit; the
# first failing step ends the call (no retries).  Outputs under gpurun_out/<tag>/.
#   bash tools/gpu_steps.sh <tag> <step> [<step> ...]
# steps:
#   tests              pytest -m gpu (the whole GPU suite)
#   tests=<expr>       pytest -m gpu -k <expr>
#   smoke              __graft_entry__.smoke()
#   driver[=cfg]       bench.py --steps 20 --warmup 5 (the driver's BENCH invocation), full line
#   quick[=cfg]        the same step counts, parity / baselines / side legs off (A/B repeats)
#   default[=cfg]      bench.py with its default step counts
#   spawn2             bench.py --gpus 2 --share-devices (bench's own rank spawner, both ranks on this GPU)
#   torchrun2          the same two ranks under python -m torch.distributed.run
#   prof=cfg           rocprofv3 --kernel-trace --stats of a 20-step bench run -> <tag>/prof_<cfg>
#   pmc=cfg            tools/pmc_kernels.sh (one rocprofv3 --pmc pass per counter group)
#   profopen=cfg       rocprofv3 --kernel-trace --stats of a short bench run with the open leg -> <tag>/profopen_<cfg>
#   pmcopen=cfg        tools/pmc_kernels.sh with the open leg -> profiles/pmc_open_<cfg>.json
#   ab=cfg:rounds:v1,v2,...   tools/ab_bench.sh (variant "base" = the product library)
#   pmclib=cfg:variant tools/pmc_kernels.sh with an experiment library -> profiles/pmc_<cfg>_<variant>.json
#   openab=cfg:rounds:v1,v2,... the open-path rate (bench's open leg, 20 + 5 seal steps) per
#                      library build, same call ("base" = the product library)
#   opensplit=cfg:rounds:m1,m2,...  the open leg with each forced split form (auto/chains/blocks/none)
#   warm               cfg2 value against warmup / timed step counts
#   mb=<mode>          tools/aes_layout_mb.bin 1027 <mode> (the AES layout microbenchmark; "t": convoy trace)
#   decmb              tools/aes_dec_mb.bin (the open path's decrypt round loop variants)
#   ldsmb              tools/lds_rate_mb.bin (LDS read rate per CU by read width and waves)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:?tag}
shift
O=$R/gpurun_out/$TAG
mkdir -p $O
QUIET="--no-cpu --no-check --no-open --no-derive --no-host-inclusive"

summ() {  # one line per bench JSON
  python3 - "$1" <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d.get("roofline") or {}
print(d["config"]["workload"][:40], "n_gpus", d["n_gpus"], "value", d["value"], "ms/step", d["ms_per_step"],
      "kernel", r.get("kernel"), r.get("kernel_avg_ms"), "frac", r.get("frac"), "traffic", r.get("traffic"),
      "bit_exact", d.get("bit_exact"), "timed", d.get("timed_bit_exact"), d.get("timed_oracle_exact"),
      "cpu", (d.get("cpu_baseline") or {}).get("value"))
EOF
}

run() {  # run <name> <limit> <cmd...>: stdout -> <name>.json / .log, stderr -> <name>.err
  local name=$1 lim=$2
  shift 2
  timeout -k 10 $lim "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "STEP $name FAILED rc=$rc"
    tail -30 $O/$name.err
    tail -5 $O/$name.out
    exit 1
  fi
}

for step in "$@"; do
  key=${step%%=*}
  arg=""
  [ "$key" != "$step" ] && arg=${step#*=}
  case $key in
    tests)
      if [ -n "$arg" ]; then
        run tests_$(echo $arg | tr -c 'A-Za-z0-9' '_') 900 python -u -m pytest tests -m gpu -k "$arg" -x -v --timeout 240 --timeout-method thread
      else
        run tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
      fi
      tail -1 $O/tests*.out ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
      tail -1 $O/smoke.out ;;
    driver)
      c=${arg:-cfg2}; n=driver_$c; i=1
      while [ -e $O/$n.out ]; do i=$((i+1)); n=driver_${c}_$i; done
      run $n 400 python bench.py --config $c --steps 20 --warmup 5
      summ $O/$n.out ;;
    quick)
      c=${arg:-cfg2}; n=quick_$c; i=1
      while [ -e $O/$n.out ]; do i=$((i+1)); n=quick_${c}_$i; done
      run $n 300 python bench.py --config $c --steps 20 --warmup 5 $QUIET
      summ $O/$n.out ;;
    default)
      c=${arg:-cfg2}
      run default_$c 600 python bench.py --config $c
      summ $O/default_$c.out ;;
    spawn2)
      run spawn2 400 python bench.py --gpus 2 --share-devices --steps 20 --warmup 5
      summ $O/spawn2.out ;;
    torchrun2)
      run torchrun2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
          --master-port 29533 bench.py --gpus 2 --share-devices --steps 20 --warmup 5
      summ $O/torchrun2.out ;;
    prof)
      c=${arg:-cfg2}; st=20; [ $c = cfg4 ] && st=3
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run \
          --output-format csv -- python3 $R/bench.py --config $c $QUIET --steps $st --warmup 1 > $O/prof_$c.out 2> $O/prof_$c.err ) \
        || { echo "STEP prof $c FAILED"; tail -20 $O/prof_$c.err; exit 1; }
      f=$(find $O/prof_$c -name "*kernel_stats.csv" | head -1)
      head -4 $f | cut -c1-200 ;;
    profopen)
      c=${arg:-cfg2}
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/profopen_$c -o run \
          --output-format csv -- python3 $R/bench.py --config $c --no-cpu --no-check --no-derive --no-host-inclusive \
          --steps 20 --warmup 5 > $O/profopen_$c.out 2> $O/profopen_$c.err ) \
        || { echo "STEP profopen $c FAILED"; tail -20 $O/profopen_$c.err; exit 1; }
      f=$(find $O/profopen_$c -name "*kernel_stats.csv" | head -1)
      head -12 $f | cut -c1-160 ;;
    pmcopen)
      c=${arg:-cfg2}
      PMC_NAME=pmc_open_$c timeout -k 10 1000 bash tools/pmc_kernels.sh $c $O/pmcopen_$c --open > $O/pmcopen_$c.log 2>&1 \
        || { echo "STEP pmcopen $c FAILED"; tail -20 $O/pmcopen_$c.log; exit 1; }
      cp $R/profiles/pmc_open_$c.json $O/pmc_open_$c.json
      python3 -c "
import json;d=json.load(open('$O/pmc_open_$c.json'))
for k,v in d['kernels'].items():
  if k.startswith('open_'): print(k, round(v.get('duration_ms',0),3), 'hbm', v.get('hbm_bytes'), 'lds_busy', v.get('lds_busy'), 'clk', v.get('clock_ghz'), 'conf', v.get('SQ_LDS_BANK_CONFLICT'), 'lds', v.get('SQ_INSTS_LDS'))
print('open call', d.get('open_call_hbm_bytes'))" ;;
    pmc)
      c=${arg:-cfg2}
      timeout -k 10 1000 bash tools/pmc_kernels.sh $c $O/pmc_$c > $O/pmc_$c.log 2>&1 \
        || { echo "STEP pmc $c FAILED"; tail -20 $O/pmc_$c.log; exit 1; }
      cp $R/profiles/pmc_$c.json $O/pmc_$c.json
      python3 -c "
import json;d=json.load(open('$O/pmc_$c.json'));k=d['dominant_kernel'];v=d['kernels'][k];print('$c', k, round(v['duration_ms'],3), 'hbm', v['hbm_bytes'], 'call', d['seal_call_hbm_bytes'])" ;;
    pmclib)  # pmclib=cfg:variant -- tools/pmc_kernels.sh with tools/ab/<variant>/libtlsgpu.so
      IFS=: read c v <<< "$arg"
      TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so PMC_NAME=pmc_${c}_$v timeout -k 10 1000 bash tools/pmc_kernels.sh $c $O/pmc_${c}_$v \
          > $O/pmc_${c}_$v.log 2>&1 || { echo "STEP pmclib $c $v FAILED"; tail -20 $O/pmc_${c}_$v.log; exit 1; }
      cp $R/profiles/pmc_${c}_$v.json $O/
      python3 -c "
import json;d=json.load(open('$O/pmc_${c}_$v.json'))
for k,v in d['kernels'].items():
    if v.get('hbm_bytes',0)>1e8: print('$c $v', k[:36], round(v['duration_ms'],3), 'read', v.get('read_bytes'), 'hbm', v['hbm_bytes'])
print('call', d['seal_call_hbm_bytes'])" ;;
    ab)
      IFS=: read c rounds variants <<< "$arg"
      timeout -k 10 1100 bash tools/ab_bench.sh gpurun_out/$TAG/ab_$c $c $rounds ${variants//,/ } \
        || { echo "STEP ab FAILED"; exit 1; } ;;
    openab)
      IFS=: read c rounds variants <<< "$arg"
      for i in $(seq 1 $rounds); do
        for v in ${variants//,/ }; do
          if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so; fi
          run openab_${c}_${v}_$i 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu --no-check --no-host-inclusive --no-derive
          python3 -c "import json;d=json.loads([l for l in open('$O/openab_${c}_${v}_$i.out') if l.startswith('{')][-1]);o=d['open'];print('$c $v open', o['value'], o['ms'], o.get('roundtrip_exact'), 'seal', d['value'])"
        done
      done
      unset TLSGPU_LIB ;;
    opensplit)
      IFS=: read c rounds modes <<< "$arg"
      for i in $(seq 1 $rounds); do
        for m in ${modes//,/ }; do
          run opensplit_${c}_${m}_$i 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu --no-check --no-host-inclusive --no-derive --open-split $m
          python3 -c "import json;d=json.loads([l for l in open('$O/opensplit_${c}_${m}_$i.out') if l.startswith('{')][-1]);o=d['open'];print('$c $m open', o['value'], o['ms'], o.get('roundtrip_exact'))"
        done
      done ;;
    ldsmb)
      run ldsmb 300 ./tools/lds_rate_mb.bin 20000
      cat $O/ldsmb.out ;;
    decmb)
      run decmb 300 ./tools/aes_dec_mb.bin 256
      cat $O/decmb.out ;;
    mb)
      run mb_${arg:-all} 300 ./tools/aes_layout_mb.bin 1027 ${arg}
      cat $O/mb_${arg:-all}.out ;;
    warm)
      for ws in "5 20" "5 50" "500 50" "500 500"; do
        set -- $ws
        run warm_w$1_s$2 300 python bench.py --config cfg2 $QUIET --warmup $1 --steps $2
        echo "warmup $1 steps $2: $(summ $O/warm_w$1_s$2.out)"
      done ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "ALL STEPS OK"
