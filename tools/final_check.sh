#!/bin/bash
# Round-end check on the GPU box (from the repo root): the full GPU suite, the
# smoke test, then tools/round_measure.sh (profiles, PMC traffic, bench lines).
set -o pipefail
R=${1:-r03}
mkdir -p gpurun_out/final
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/final/gputest.log 2>&1 || { echo "GPU suite failed"; tail -40 gpurun_out/final/gputest.log; exit 1; }
tail -1 gpurun_out/final/gputest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 \
    || { echo "smoke failed"; cat gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 1100 bash tools/round_measure.sh "$R" || { echo "round_measure failed"; exit 1; }
echo "final check done"
