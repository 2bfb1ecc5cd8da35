#!/bin/bash
# Round-end rehearsal on the final tree: GPU tests, smoke, the default bench and the
# driver's bench invocation (--steps 20 --warmup 5).  Each step under its own limit;
# the first failure ends the run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_check
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  && timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
  && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
rc=$?
tail -2 $O/pytest.log
cat $O/smoke.log $O/bench_default.json $O/bench_driver.json 2>/dev/null
exit $rc
