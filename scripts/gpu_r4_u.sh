#!/bin/bash
# closing-tree counters: config 2 and config 4 traces + three PMC passes each.
bash "$(dirname "$0")/gpu_r4_pmc.sh" 2 && bash "$(dirname "$0")/gpu_r4_pmc.sh" 4
