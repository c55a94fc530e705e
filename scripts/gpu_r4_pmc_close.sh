#!/bin/bash
# closing-tree counters: configs 2 and 4 (trace + three pmc passes each)
bash "$(dirname "$0")/gpu_r4_pmc.sh" 2 && bash "$(dirname "$0")/gpu_r4_pmc.sh" 4
