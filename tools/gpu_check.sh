#!/bin/bash
# smoke -> pytest -m gpu -> short bench, each step under its own time limit;
# stops at the first step that faults, aborts or times out.
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
