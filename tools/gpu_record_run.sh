#!/bin/bash
# The record run of a round on one MI355X (tools/gpu_steps.sh steps): the GPU suite, smoke,
# every config at the driver's step counts (20 + 5) and at bench.py's defaults, the N = 2
# launch paths (bench's own rank spawner and torch.distributed.run, both ranks on this box's
# one GPU: the launch contract, not a scaling number), rocprofv3 kernel statistics and PMC
# passes of every config.  Stops at the first failure.
#   bash tools/gpu_record_run.sh <tag> [steps...]     (outputs under gpurun_out/<tag>)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:-record}
shift
STEPS="$@"
[ -z "$STEPS" ] && STEPS="tests smoke driver driver default driver=cfg3 default=cfg3 default=cfg4 driver=cfg5 default=cfg5 \
spawn2 torchrun2 prof=cfg2 prof=cfg3 prof=cfg4 prof=cfg5 pmc=cfg2 pmc=cfg3 pmc=cfg4 pmc=cfg5"
bash tools/gpu_steps.sh $TAG $STEPS
