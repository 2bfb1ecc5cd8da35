R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for s in 0 2; do
TLSGPU_DEBUG_SKIP=$s timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/pmc_a$s -o run -- python $R/bench.py --steps 3 --warmup 1 --no-check --no-cpu > $R/gpurun_out/pmc_a$s.log 2>&1 || exit 1
TLSGPU_DEBUG_SKIP=$s timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/pmc_b$s -o run -- python $R/bench.py --steps 3 --warmup 1 --no-check --no-cpu > $R/gpurun_out/pmc_b$s.log 2>&1 || exit 1
done
ls -R $R/gpurun_out/pmc_a0 | head
