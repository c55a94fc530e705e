#!/bin/bash
# Re-entry check: GPU tests, smoke(), headline bench.
source "$(dirname "$0")/gpu_round.sh"
run gputests 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 30 --warmup 5
