#!/bin/bash
# re-entry check after a rebuilt extension: smoke, the default bench, GPU suite, configs 2-5, config-2 kernel profile
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 600 python bench.py
bash "$(dirname "$0")/gpu_final.sh"
